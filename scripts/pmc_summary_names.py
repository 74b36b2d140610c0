"""Kernel names as the engine reports them (fdbcs_kernel_profile)."""


def engine_name(n: str) -> str:
    n = n.strip()
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):  # cut the parameter list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            n = n[:i]
            break
    return n[len("fdbcs::"):] if n.startswith("fdbcs::") else n
