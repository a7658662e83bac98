"""GPU: the seeded closed-loop regression harness (tests/sim_regress.py) for each model: multi-tick warm-start
chain with seeded resets, every check tick replayed through the fp64 oracle (|u0 - u0_oracle| <= 1e-3, the same
solve statuses, no failed solve)."""
import pytest

from tests.sim_regress import run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,N,B", [("diff", 40, 1024), ("omni4", 30, 512), ("tric", 40, 512)])
def test_closed_loop_regression(built, model, N, B):
    rep = run(model, N, B, ticks=30, sample=48, check_every=5, reset_frac=0.05, reset_every=4)
    assert rep["failed"] == 0
    assert rep["resets"] > 0 and len(rep["checks"]) == 6
    assert all(c["status_mismatch"] == 0 and c["oracle_failed"] == 0 for c in rep["checks"]), rep["checks"]
    assert rep["u0_err_max"] <= 1e-3 and rep["cmd_err_max"] <= 1e-3, rep["checks"]
