"""The multi-GPU bench path, rehearsed on one GPU: two ranks (gloo, since RCCL refuses two ranks
on one card) each resolve their key-range shard with the HIP engine, scatter conflict bytes on
the device and all-reduce them; every rank's verdicts must equal its own CPU restatement fed the
same routing, and the device-side combine must equal the host-built one."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("workload,extra", [("c2", []), ("c3", []), ("c3", ["--reshard", "--reshard-preroll", "60"])])
def test_two_rank_bench_parity(engine, workload, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--workload", workload, "--steps", "8", "--warmup", "2", "--txns", "1000",
           "--history", "200000", "--resident-steps", "0", "--total-steps", "0", "--breakdown-steps", "0",
           "--profile-steps", "4", "--sync-steps", "4", "--backend", "gloo", "--cpu-seconds", "20"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, "\n".join([l for l in r.stderr.splitlines() if "[rank1]" in l][-30:]) + r.stderr[-1500:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0
    # warmup 2 + profile 4 + timed 8 + sync 4 batches, every one combined and replayed on each rank
    assert out["parity"]["batches_checked"] >= 2 * 18 and out["parity"]["mismatched_batches"] == 0
    assert out["combine_check"]["mismatched"] == 0 and out["combine_check"]["batches"] == 18
    # G resolvers on G cores: both ranks' restatements timed at once, over the slower one
    assert out["cpu_baseline"]["cores"] == 2 and out["cpu_baseline"]["value"] > 0
    assert out["distributed"]["world_size"] == 2 and out["distributed"]["backend"] == "gloo"
    assert out["combine_check"]["path"].startswith("device conflict bytes")
    if extra:
        assert out["reshard"]["moves"] > 0  # the hot rank gave key ranges away
