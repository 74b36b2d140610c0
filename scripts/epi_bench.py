"""Isolated cost of the whole-tier index rebuild (k_epilogue<true> via fdbcs_load_history's
launch_rangemax) on a C2 history: run under rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.is_available()
from foundationdb_amd import conflict_set as C  # noqa: E402
from foundationdb_amd import workloads as W  # noqa: E402

p = W.C2Params(history=int(os.environ.get("HISTORY", 5_000_000)))
kb, ko, vers = W.c2_history(p, seed=1, start_version=10_000_000)
cs = C.ConflictSet(0)
for _ in range(int(os.environ.get("REPS", 5))):
    cs.load_history(kb, ko, vers, 0)
print("loaded", cs.history_size())
cs.close()
