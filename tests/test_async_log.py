"""Loss readback without per-step host syncs (engine/trainer.py AsyncLossLog,
the process_epoch / train.py logging path; reference: train.py:175-180 prints
float(loss) every step)."""
import pytest
import torch

from ncnet_amd.engine.trainer import AsyncLossLog


def test_cpu_log_is_immediate_and_ordered():
    log = AsyncLossLog("cpu")
    assert log.sync
    recs = []
    for i in range(5):
        recs += log.push(torch.tensor(float(i)), {"step": i})
    recs += log.drain()
    assert [r["step"] for r in recs] == list(range(5))
    assert [r["loss"] for r in recs] == [float(i) for i in range(5)]
    assert all(r["elapsed_s"] >= 0 for r in recs)


@pytest.mark.gpu
def test_gpu_log_async_in_order_and_complete():
    log = AsyncLossLog("cuda")
    assert not log.sync
    x = torch.randn(2048, 2048, device="cuda")
    recs = []
    want = []
    for i in range(8):
        y = x @ x                      # keep the stream busy: pushes must not wait for it
        v = y[0, 0] * 0 + i
        want.append(float(i))
        recs += log.push(v, {"step": i})
    recs += log.drain()
    assert [r["step"] for r in recs] == list(range(8))
    assert [r["loss"] for r in recs] == want
    el = [r["elapsed_s"] for r in recs]
    assert el == sorted(el) and el[0] > 0
