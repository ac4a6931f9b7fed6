"""bench/calibrate.py: the box-speed record of bench.py (sysfs clock / power
parsing on a fake device tree; off the GPU the record is absent)."""
import time

import torch

from tf_operator_amd.bench import calibrate


def _dev(tmp_path, hwmon_freq=None, dpm=None, power=None, busy=None):
    d = tmp_path / "device"
    hw = d / "hwmon" / "hwmon3"
    hw.mkdir(parents=True)
    if hwmon_freq is not None:
        (hw / "freq1_input").write_text(str(hwmon_freq))
        (hw / "freq1_label").write_text("sclk")
    if dpm is not None:
        (d / "pp_dpm_sclk").write_text(dpm)
    if power is not None:
        (hw / "power1_average").write_text(str(power))
    if busy is not None:
        (d / "gpu_busy_percent").write_text(str(busy))
    return str(d)


def test_sclk_prefers_hwmon_then_active_dpm_level(tmp_path):
    d = _dev(tmp_path, hwmon_freq=1_742_000_000, dpm="0: 500Mhz\n1: 1700Mhz *\n2: 2400Mhz\n")
    assert calibrate.read_sclk_mhz(d) == (1742.0, "hwmon freq1_input")
    d2 = _dev(tmp_path / "b", dpm="0: 500Mhz\n1: 1700Mhz *\n2: 2400Mhz\n")
    assert calibrate.read_sclk_mhz(d2) == (1700.0, "pp_dpm_sclk")
    assert calibrate.read_sclk_mhz(str(tmp_path / "none")) == (None, "unavailable")


def test_sampler_summarises_clock_power_busy(tmp_path):
    d = _dev(tmp_path, hwmon_freq=2_000_000_000, power=750_000_000, busy=97)
    s = calibrate.ClockSampler(d, period_s=0.01).start()
    time.sleep(0.08)
    out = s.stop()
    assert out["samples"] >= 2 and out["gfxclk_mhz_mean"] == 2000.0 and out["gfxclk_mhz_min"] == 2000.0
    assert out["power_w_mean"] == 750.0 and out["busy_pct_mean"] == 97.0
    assert calibrate.ClockSampler(None).start().stop() == {}


def test_calibration_is_absent_off_the_gpu():
    c = calibrate.Calibration(torch.device("cpu"))
    c.before()
    c.start()
    c.stop()
    c.after()
    assert c.record() is None


def test_record_means_of_before_and_after():
    c = calibrate.Calibration(torch.device("cpu"))
    c.on = True
    c.rec = {"before": {"hipblaslt_pfs": 1.5, "asm_pfs": 1.4}, "after": {"hipblaslt_pfs": 1.3, "asm_pfs": 1.4}}
    r = c.record()
    assert r["gemm_shape_mnk"] == [8192, 8192, 8192]
    assert r["hipblaslt_pfs_mean"] == 1.4 and r["asm_pfs_mean"] == 1.4
