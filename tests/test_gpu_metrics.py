"""Per-pod GPU device metrics (utils/gpu_metrics.py): the cAdvisor
accelerator series of the reference's monitoring guide
(docs/monitoring/README.md:26-29) for MI355X, read from amdgpu sysfs and
attributed to the pods the local kubelet gave each device."""
import json
import os
import sys

from tf_operator_amd.sdk import container, pod_template
from tf_operator_amd.testing.cluster import LocalCluster
from tf_operator_amd.utils import gpu_metrics

HERE = os.path.dirname(os.path.abspath(__file__))


def _fake_sysfs(root, n=2):
    """amdgpu sysfs layout: cardN/device/{mem_info_vram_*, gpu_busy_percent, hwmon/hwmonK/*}."""
    for i in range(n):
        d = os.path.join(root, f"card{i}", "device")
        hw = os.path.join(d, "hwmon", f"hwmon{3 + i}")
        os.makedirs(hw)
        files = {"mem_info_vram_total": 309220868096, "mem_info_vram_used": (i + 1) * 10 << 30,
                 "gpu_busy_percent": 40 + i}
        for k, v in files.items():
            with open(os.path.join(d, k), "w") as f:
                f.write(f"{v}\n")
        for k, v in {"power1_average": 750_000_000 + i, "temp1_input": 46000, "temp1_label": "junction"}.items():
            with open(os.path.join(hw, k), "w") as f:
                f.write(f"{v}\n")
    # a display-only card without VRAM and a connector node are skipped
    os.makedirs(os.path.join(root, f"card{n}", "device"))
    os.makedirs(os.path.join(root, "card0-DP-1"))


def test_read_devices_and_exposition(tmp_path):
    _fake_sysfs(str(tmp_path))
    devs = gpu_metrics.read_devices(str(tmp_path))
    assert [d["acc_id"] for d in devs] == ["card0", "card1"]
    assert devs[1]["memory_used_bytes"] == 20 << 30
    assert devs[0]["duty_cycle"] == 40 and abs(devs[0]["power_watts"] - 750.0) < 1e-6
    assert devs[0]["temperature_celsius"] == {"junction": 46.0}
    text = gpu_metrics.exposition(devs, {1: ("default", "job-worker-0", "tensorflow")})
    assert "# TYPE container_accelerator_memory_used_bytes gauge" in text
    assert ('container_accelerator_memory_used_bytes{make="amd",model="MI355X",acc_id="card1",'
            'namespace="default",pod="job-worker-0",container="tensorflow"} 2.14748e+10') in text
    assert 'container_accelerator_duty_cycle{make="amd",model="MI355X",acc_id="card0",namespace="",pod=""' in text
    assert 'toa_gpu_power_watts{acc_id="card0"} 750' in text


def test_from_amd_smi():
    doc = {"gpu_data": [{"gpu": 0, "usage": {"gfx_activity": {"value": 87, "unit": "%"},
                                             "umc_activity": {"value": 40, "unit": "%"}},
                         "power": {"socket_power": {"value": 1210, "unit": "W"}},
                         "temperature": {"edge": "N/A", "hotspot": {"value": 71, "unit": "C"}},
                         "ecc": {"total_uncorrectable_count": 0},
                         "mem_usage": {"total_vram": {"value": 294896, "unit": "MB"},
                                       "used_vram": {"value": 248000, "unit": "MB"}}}]}
    d = gpu_metrics.from_amd_smi(doc)[0]
    assert d["duty_cycle"] == 87 and d["umc_activity"] == 40 and d["power_watts"] == 1210
    assert d["memory_used_bytes"] == 248000 * (1 << 20) and d["temperature_celsius"] == {"hotspot": 71}
    assert "container_accelerator_memory_total_bytes" in gpu_metrics.exposition([d])


def test_kubelet_attributes_devices_to_pods(tmp_path):
    """A running 2-worker TFJob holding virtual amd.com/gpu devices 0 and 1:
    the node's accelerator series name the pods."""
    _fake_sysfs(str(tmp_path), n=3)
    cmd = [sys.executable, "-c", "import time; time.sleep(30)"]
    tpl = pod_template(container(image="toa/trainer", command=cmd, gpus=1, env={"TOA_NO_GPU": "1"}))
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": "gm", "namespace": "default"},
           "spec": {"runPolicy": {"cleanPodPolicy": "All"},
                    "tfReplicaSpecs": {"Worker": {"replicas": 2, "restartPolicy": "Never", "template": tpl}}}}
    with LocalCluster(gpus=3) as c:
        c.client.create(job)
        c.wait(lambda: len(c.kubelet.gpu_owners()) == 2, 30, 0.05, "pods bound to GPUs")
        text = c.gpu_metrics_text(str(tmp_path))
        owners = c.kubelet.gpu_owners()
        assert {v[1] for v in owners.values()} == {"gm-worker-0", "gm-worker-1"}
        for idx, (_, pod, _) in owners.items():
            assert f'acc_id="card{idx}",namespace="default",pod="{pod}",container="tensorflow"' in text
        assert text.count('pod=""') == 3  # the free device: memory used / total / duty cycle
        c.client.delete("gm")
    assert json.loads(json.dumps(owners))  # serialisable for the --owners file of the exporter


def test_read_devices_accessible_only(tmp_path):
    """A shared host: sysfs lists every card, /dev/dri only this process's
    render node (card1's here) -- accessible_only keeps just that GPU."""
    root = str(tmp_path / "drm")
    _fake_sysfs(root)
    os.makedirs(os.path.join(root, "renderD129"))
    os.symlink(os.path.join(root, "card1", "device"), os.path.join(root, "renderD129", "device"))
    dri = tmp_path / "dri"
    dri.mkdir()
    (dri / "renderD129").write_text("")
    devs = gpu_metrics.read_devices(root, accessible_only=True, dev_dri=str(dri))
    assert [d["acc_id"] for d in devs] == ["card1"] and devs[0]["index"] == 0
    assert len(gpu_metrics.read_devices(root)) == 2
