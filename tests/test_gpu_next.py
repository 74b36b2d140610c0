"""§8(f) rows on the GPU engine: dynamic resharding (ownership-history routing, the balancer) and
the cross-resolver conflicting-key remap over several engine instances, checked bit-exact
against oracles fed the same routing; client-produced transactions resolved by the engine keep
read-modify-write serializable."""
import numpy as np
import pytest

from foundationdb_amd import balancing as B
from foundationdb_amd import client as CL
from foundationdb_amd import workloads as W
from foundationdb_amd.packing import PackedBatch
from foundationdb_amd.sharding import KeyResolvers, KeyRangeSharding, combine, combine_conflicting_keys
from tests.helpers import EngineDriver

pytestmark = pytest.mark.gpu


def _sorted(conf):
    return {t: sorted(v) for t, v in conf.items()}


def test_resharded_engines_match_resharded_oracles(engine, oracle_built):
    """Three engines behind KeyResolvers whose map moves every few batches: per-resolver verdicts
    and reports, the min combine and the proxy's remapped conflicting keys all equal the oracles'."""
    G = 3
    kr = KeyResolvers(G, [bytes([85]), bytes([170])])
    engines = [EngineDriver(engine) for _ in range(G)]
    oracles = [oracle_built.OracleConflictSet() for _ in range(G)]
    rng = np.random.default_rng(31)
    now = 10
    reported = 0
    for i in range(18):
        if i % 3 == 1:
            a = int(rng.integers(0, 250))
            kr.apply_changes([(bytes([a]), bytes([min(255, a + int(rng.integers(5, 60)))]), int(rng.integers(0, G)))], now)
        pb = W.random_small_batch(rng, 300, alphabet=256, max_len=3, now=now, staleness=12, report_frac=0.5)
        parts = kr.route(pb)
        re = [engines[g].detect(parts[g].batch, now, now - 9) for g in range(G)]
        ro = [oracles[g].detect(parts[g].batch, now, now - 9) for g in range(G)]
        for g in range(G):
            assert (re[g][0] == ro[g][0]).all()
            assert _sorted(re[g][1]) == _sorted(ro[g][1])
        v = combine(pb.n_txn, parts, [r[0] for r in re])
        assert (v == combine(pb.n_txn, parts, [r[0] for r in ro])).all()
        ke = combine_conflicting_keys(pb, parts, [_sorted(r[1]) for r in re], v)
        ko = combine_conflicting_keys(pb, parts, [_sorted(r[1]) for r in ro], v)
        assert ke == ko
        reported += sum(len(x) > 0 for x in ke.values())
        if i % 6 == 5:
            kr.coalesce(now, life_versions=20)
        now += 3
    assert reported > 20


def test_balancer_over_engines_on_hot_keys(engine, oracle_built):
    """The balancer moves load under Zipf-skewed keys (C3 shape, small) while two engines keep
    matching two oracles fed the same (changing) routing."""
    G = 2
    p = W.C2Params(txns=400)
    zipf = W.ZipfGenerator(100_000)
    br = B.BalancedRouting(G, KeyResolvers.from_sharding(KeyRangeSharding.uniform(G)), seed=3,
                           min_balance_difference=5_000, balance_time=0.005, key_bytes_per_sample=1_000)
    engines = [EngineDriver(engine) for _ in range(G)]
    oracles = [oracle_built.OracleConflictSet() for _ in range(G)]
    rng = np.random.default_rng(5)
    version = 10_000_000
    for _ in range(40):
        pb = W.c3_batch(p, rng, version, zipf)
        parts = br.route(pb, version)
        for g in range(G):
            ve, _ = engines[g].detect(parts[g].batch, version, version - 5_000_000)
            vo, _ = oracles[g].detect(parts[g].batch, version, version - 5_000_000)
            assert (ve == vo).all()
        version += 1000
    assert br.balancer.moves_made > 0


def test_client_increments_on_engine(engine):
    """Read-modify-write counters produced through the client Transaction API and resolved by the
    HIP engine: every committed increment is reflected exactly once."""
    from tests.test_client import _run_increments

    drv = EngineDriver(engine)

    def resolve(pb, now, no):
        return drv.detect(pb, now, no)[0]

    store, committed = _run_increments(resolve, n_clients=40, rounds=30)
    for k in range(len(committed)):
        assert int.from_bytes(store.read(b"ctr%d" % k, store.version), "little") == committed[k]
    assert 0 < committed.sum() < 40 * 30


def test_device_conflict_output(engine):
    """fdbcs_batch_set_conflict_output: detect also writes 2 - verdict at each routed transaction's
    global index (0 elsewhere) into torch-allocated device memory, complete when the batch is:
    the input of the multi-GPU MAX all-reduce (bench.py)."""
    import torch

    sh = KeyRangeSharding.uniform(2)
    rng = np.random.default_rng(41)
    cs = engine.ConflictSet(0)
    now = 10
    for _ in range(6):
        pb = W.random_small_batch(rng, 400, alphabet=256, max_len=3, now=now, staleness=10)
        part = sh.route(pb)[1]
        out = torch.full((pb.n_txn,), 7, dtype=torch.uint8, device="cuda")  # every byte is written
        torch.cuda.synchronize()  # torch's fill is on torch's stream: finish it before the engine writes
        b = engine.ConflictBatch(cs)
        b.add_packed(part.batch)
        b.set_conflict_output(part.txn_ids, pb.n_txn, out.data_ptr())
        b.detect_async(now, now - 5)
        v = b.wait()
        b.close()
        want = KeyRangeSharding.conflict_bytes(pb.n_txn, part, v)
        assert np.array_equal(out.cpu().numpy(), want)
        now += 3
    cs.close()
