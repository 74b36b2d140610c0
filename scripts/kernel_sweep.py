"""Device time of pipeline kernels alone (fdbcs_debug_kernel_time) on a full-size workload, under
the env-knob variants given on the command line ("FDBCS_CHECK=1", "FDBCS_SORT_WIN=0"...).  WHICH
lists the kernels (0 read check, 1 sample, 2 bucket count, 3 scatter, 4 bucket sort; default 0).
Each variant runs in a fresh subprocess (knobs are read when a conflict set is created)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(workload):
    sys.path.insert(0, ROOT)
    import numpy as np

    from foundationdb_amd import conflict_set as C
    from foundationdb_amd import workloads as W

    start = 10_000_000
    if workload == "c4":
        p = W.C4Params(history=int(os.environ.get("HISTORY", 50_000_000)))
        kb, ko, vers = W.c4_history(p, seed=1000, start_version=start)
        mk = lambda rng, now: W.c4_batch(p, rng, now)
    else:
        p = W.C2Params(history=int(os.environ.get("HISTORY", 5_000_000)), txns=int(os.environ.get("TXNS", 5000)))
        kb, ko, vers = W.c2_history(p, seed=1, start_version=start)
        z = W.ZipfGenerator(1_000_000, 0.99) if workload == "c3" else None
        mk = (lambda rng, now: W.c3_batch(p, rng, now, z)) if z else (lambda rng, now: W.c2_batch(p, rng, now))
    cs = C.ConflictSet(0)
    cs.load_history(kb, ko, vers, 0)
    rng = np.random.default_rng(5)
    now = start
    out = []
    for i in range(6):  # a few real batches first so the delta tier is populated
        now += 1000
        b = C.ConflictBatch(cs)
        b.add_packed(mk(rng, now))
        b.detect_conflicts(now, now - p.window)
        b.close()
    for i in range(3):
        b = C.ConflictBatch(cs)
        b.add_packed(mk(rng, now + 1000))
        which = [int(x) for x in os.environ.get("WHICH", "0").split(",")]
        out.append({w: round(b.debug_kernel_time(w, 40), 1) for w in which})
        b.close()
    return out


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        print(json.dumps(one(sys.argv[2])))
        sys.exit(0)
    workload = os.environ.get("WORKLOAD", "c2")
    for spec in sys.argv[1:]:
        env = dict(os.environ)
        env.pop("WORKLOAD", None)
        for kv in spec.split():
            if "=" in kv:
                k, v = kv.split("=", 1)
                env[k] = v
        r = subprocess.run([sys.executable, __file__, "--one", workload], env=env, capture_output=True, text=True,
                           timeout=300)
        if r.returncode:
            print(spec, "FAILED", r.stderr[-2000:], flush=True)
            sys.exit(r.returncode)
        w = env.get("WORKLOAD_OVERRIDE", workload)
        print(f"{workload} {spec:40s} us: {json.loads(r.stdout.strip().splitlines()[-1])}", flush=True)
        for line in r.stderr.splitlines():
            if line.startswith("fdbcs sort"):
                print("   ", line, flush=True)
