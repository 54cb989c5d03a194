"""The pbft_replica state machine with the real GPU verifier and GPU request digest."""
import numpy as np
import pytest

from replica_sim import EV_COMMITTED, Cluster, PhaseSim
from test_replica import run_round

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_cluster():
    from pbft_amd import GpuBatchVerifier
    v = GpuBatchVerifier(0)
    yield v
    v.close()


def test_gpu_cluster_rounds(gpu_cluster):
    v = gpu_cluster
    c = Cluster(4, ctx=v._ctx, use_oracle_verifier=False)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    evs = run_round(c, seq=1)
    for r in range(4):
        assert (1, 1, EV_COMMITTED) in evs[r]
    evs = run_round(c, byzantine={3}, seq=2)
    for r in range(3):
        assert (1, 2, EV_COMMITTED) in evs[r]
    evs = run_round(c, byzantine={1, 3}, seq=3)
    assert not any(e[2] == EV_COMMITTED for r in range(4) for e in evs[r])
    c.close()


@pytest.mark.parametrize("n,silent,forgers", [(4, {3}, set()), (7, {5}, {6})])
def test_gpu_phase_ordered_rounds(gpu_cluster, n, silent, forgers):
    """Phase-ordered rounds (Commit only after PREPARED), f silent / id-forging replicas, no forced flush: every
    PrePrepare, Prepare and Commit signature is checked by the GPU kernels, digests by the GPU Blake2b."""
    v = gpu_cluster
    c = Cluster(n, ctx=v._ctx, use_oracle_verifier=False, tag=11)
    assert v.set_keys(np.frombuffer(c.keys, dtype=np.uint8)).all()
    sim = PhaseSim(c, silent=silent, forgers=forgers)
    seqs = range(1, 17)
    sim.start(1, seqs)
    assert sim.run() < 20
    for i in sim.honest():
        assert sim.committed(i, 1, seqs), (i, sim.events[i])
        st = c.stats(i)
        assert st["live_windows"] == 0 and st["low_watermark"] == 16
        if forgers:
            assert st["rejected_sig"] > 0
    c.close()
