"""The pbft_replica state machine with the real GPU verifier and GPU request digest."""
import pytest

from replica_sim import EV_COMMITTED, Cluster
from test_replica import run_round

pytestmark = pytest.mark.gpu


def test_gpu_cluster_rounds():
    from pbft_amd import GpuBatchVerifier
    v = GpuBatchVerifier(0)
    c = Cluster(4, ctx=v._ctx, use_oracle_verifier=False)
    import numpy as np
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
    v.close()
