"""The opt-in fused forward chain (CSA_FWD_CHAIN=1: fc1 forward | fc2 forward | head in one
launch with ticket hand-offs, dense_direct.hip fwd_chain_kernel) trains like the default
three launches; its bounded waits never time out."""
import pytest
import torch

from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine

pytestmark = pytest.mark.gpu


def test_fwd_chain_matches_separate_launches(monkeypatch):
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3,
                                  options={"batch_size": 50}))
    ds = synthetic_mnist(2000, seed=0)
    monkeypatch.setenv("CSA_FWD_CHAIN", "1")
    a = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    monkeypatch.setenv("CSA_FWD_CHAIN", "0")
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    assert a.program.chain and not b.program.chain
    for _ in range(4):
        a.step(); b.step()
    a.run_steps(16); b.run_steps(16)
    a.sync_device(); b.sync_device()
    assert int(a.program.chain_err.item()) == 0
    a.check_health()
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)
