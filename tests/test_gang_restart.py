"""Config #4 (gang-scheduled TFJob, restartPolicy OnFailure) recovery on the
local cluster: a SIGKILLed rank is restarted in place, the surviving ranks
leave the broken process group with the retryable peer-lost code and are
restarted too, and the group resumes training from its checkpoint
(benchmarks/gang_restart.py)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gang_onfailure_group_recovers_after_rank_kill():
    spec = importlib.util.spec_from_file_location("gang_restart", os.path.join(ROOT, "benchmarks", "gang_restart.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = mod.main(["--workers", "3", "--run-before", "2", "--timeout", "180"])
    assert out["podgroup_min_member"] == 3
    assert 0 < out["value"] < 60, out  # fault -> first step of the restarted group
    assert out["restarts"] and all(v >= 1 for v in out["restarts"].values()), out["restarts"]
    assert "Failed" not in out["conditions"], out["conditions"]
    assert out["samples_per_sec_after"] > 0
