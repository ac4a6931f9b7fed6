"""Profiling hooks: the operator wraps a replica's command with the rocprofv3
launcher when the job asks for it (annotation amd.com/rocprof), the launcher
builds a profiler command line that obeys the pool's rules, and the summary
reads rocprofv3's stats / trace CSVs."""
import os

import pytest

from tf_operator_amd import core
from tf_operator_amd.testing import fixtures as fx
from tf_operator_amd.utils import profiling

NOW = 1_700_000_000.0


def _created_pods(job):
    res = core.reconcile(job, [], [], now=NOW, options={})
    return [a["pod"] for a in res["actions"] if a["op"] == "create_pod"]


def test_rocprof_annotation_wraps_main_container():
    job = fx.new_tfjob(worker=2)
    for s in job["spec"]["tfReplicaSpecs"].values():
        s["template"]["spec"]["containers"][0]["command"] = ["python3", "-m", "trainer", "--steps", "5"]
        s["template"]["spec"]["containers"].append({"name": "sidecar", "image": "x", "command": ["sleep", "1"]})
    job["metadata"]["annotations"] = {"amd.com/rocprof": "pmc:SQ_WAVES,SQ_INSTS_MFMA", "amd.com/rocprof-dir": "/prof"}
    pods = _created_pods(job)
    assert len(pods) == 2
    for p in pods:
        main = [c for c in p["spec"]["containers"] if c["name"] == "tensorflow"][0]
        side = [c for c in p["spec"]["containers"] if c["name"] == "sidecar"][0]
        name = p["metadata"]["name"]
        assert main["command"] == ["python3", "-m", "tf_operator_amd.utils.profiling", "--mode",
                                   "pmc:SQ_WAVES,SQ_INSTS_MFMA", "--out", f"/prof/{name}", "--", "python3", "-m",
                                   "trainer", "--steps", "5"]
        assert side["command"] == ["sleep", "1"]


def test_no_annotation_or_no_command_leaves_pod_alone():
    job = fx.new_tfjob(worker=1)
    before = [c.get("command") for c in job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"]]
    assert [c.get("command") for c in _created_pods(job)[0]["spec"]["containers"]] == before
    job["metadata"]["annotations"] = {"amd.com/rocprof": "stats"}  # image entrypoint: nothing to wrap
    for c in job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"]:
        c.pop("command", None)
    assert "command" not in _created_pods(job)[0]["spec"]["containers"][0]


def test_rocprof_argv_rules():
    a = profiling.rocprof_argv(["python3", "bench.py", "--steps", "2"], "out", "stats")
    assert a[-5:] == ["--", "python3", "bench.py", "--steps", "2"] and "--stats" in a and "--kernel-trace" in a
    p = profiling.rocprof_argv(["./bench"], "out", "pmc", ["SQ_WAVES"])
    assert p[1:3] == ["--pmc", "SQ_WAVES"] and "--stats" not in p
    for banned in ("--sys-trace", "--runtime-trace", "-s", "-r"):
        assert banned not in p
    with pytest.raises(ValueError):
        profiling.rocprof_argv(["env", "X=1", "python3"], "out")  # no launcher hop under the profiler
    with pytest.raises(ValueError):
        profiling.rocprof_argv(["./bench"], "out", "pmc")


def test_summary_from_stats_and_trace(tmp_path):
    d = tmp_path / "stats"
    d.mkdir()
    (d / "run_kernel_stats.csv").write_text(
        '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
        '"gemm(int)",10,3000000,300000,75,1,1,0\n"norm(float)",5,1000000,200000,25,1,1,0\n')
    md = profiling.summarize(str(d))
    assert "| 75.0 | 3.00 | 10 | 300.0 | `gemm` |" in md
    t = tmp_path / "trace"
    t.mkdir()
    (t / "run_kernel_trace.csv").write_text(
        '"Kernel_Name","Start_Timestamp","End_Timestamp"\n"a(x)",0,1000\n"a(x)",2000,3000\n"b",0,6000\n')
    md = profiling.summarize(str(t))
    assert md.index("`b`") < md.index("`a`") and "| 2 | 1.0 |" in md


def test_launcher_runs_child_and_writes_summary(tmp_path, monkeypatch):
    """Without rocprofv3 on PATH the launcher still runs the program (as a
    child process) and returns its exit code."""
    monkeypatch.setenv("PATH", "/usr/bin:/bin")
    if os.path.exists("/opt/rocm/bin/rocprofv3"):
        pytest.skip("rocprofv3 present: the unprofiled fallback is not reachable")
    rc = profiling.main(["--out", str(tmp_path), "--", "python3", "-c", "import sys; sys.exit(3)"])
    assert rc == 3


def test_launcher_command_is_left_unwrapped_with_warning():
    """A shell/launcher first (bare or by path) is never wrapped: the hop would
    re-exec under rocprofv3's preload.  The core emits a Warning instead."""
    for argv0 in ("bash", "/bin/sh", "/usr/bin/env"):
        job = fx.new_tfjob(worker=1)
        c = job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]
        c["command"] = [argv0, "-c", "python3 train.py"]
        job["metadata"]["annotations"] = {"amd.com/rocprof": "stats"}
        res = core.reconcile(job, [], [], now=NOW, options={})
        pod = [a["pod"] for a in res["actions"] if a["op"] == "create_pod"][0]
        assert pod["spec"]["containers"][0]["command"] == [argv0, "-c", "python3 train.py"]
        assert any(e["reason"] == "RocprofSkipped" for e in res["events"]), res["events"]
    with pytest.raises(ValueError):
        profiling.rocprof_argv(["/usr/bin/env", "python3"], "out")


def test_launcher_falls_back_to_unprofiled_run_for_launcher_hop(tmp_path, monkeypatch):
    monkeypatch.setattr(profiling.shutil, "which", lambda n: "/opt/rocm/bin/rocprofv3")
    rc = profiling.main(["--out", str(tmp_path), "--", "/bin/sh", "-c", "exit 7"])
    assert rc == 7
