"""bench.py's cpu_baseline leg parses the reference CLI's `[persistent]` lines
(c/main.c:262-271), which the reference prints only for --benchmark-runs > 1
(c/main.c:263-264): the 16-thread row (3 runs) and the 1-thread row (2 runs,
2 frames) both ask for >= 2 runs, and the 128-frame extrapolation follows the
median run.  The reference itself is replaced by a recorded stderr here (no
GPU, no minutes of CPU decode)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _stderr(runs, frames, talker_ms, codec_ms, total_ms):
    lines = ["Codec decode complete: 3840 samples (0.16 seconds)"]
    for i in range(runs):
        lines.append(f"[persistent] run {i + 1}/{runs}: elapsed={total_ms[i]:.1f} ms, audio={frames * 0.08:.2f}s, "
                     f"talker={talker_ms[i]:.1f} ms, codec={codec_ms[i]:.1f} ms, total={total_ms[i]:.1f} ms, "
                     f"tokens={frames}")
    return "\n".join(lines) + "\n"


def test_cpu_baseline_parses_runs_and_extrapolates(monkeypatch, tmp_path):
    exe = tmp_path / "oracle" / "_ref" / "qwen-tts"
    exe.parent.mkdir(parents=True)
    exe.write_text("")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    seen = {}

    def fake_run(cmd, env=None, capture_output=True, text=True, timeout=None):
        seen["cmd"], seen["threads"] = cmd, env["OMP_NUM_THREADS"]
        runs = int(cmd[cmd.index("--benchmark-runs") + 1])
        frames = int(cmd[cmd.index("--fixed-codec-tokens") + 1])
        err = _stderr(runs, frames, [1000.0 * frames + 10 * i for i in range(runs)], [100.0 * frames] * runs,
                      [7000.0 + 1100.0 * frames + 10 * i for i in range(runs)])
        return subprocess.CompletedProcess(cmd, 0, "", err)

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    r = bench.cpu_baseline("/m", [1, 2, 3], 16, frames=8, warmup=1, runs=3, target_frames=128)
    assert r is not None and r["cores"] == 16 and seen["threads"] == "16" and len(r["runs"]) == 3
    # median run: fixed 7000 ms + (talker 8010 + codec 800) / 8 per frame x 128
    med_talker, med_total = 8010.0, 7000.0 + 8800.0 + 10.0
    fixed = med_total - med_talker - 800.0
    ext = fixed + (med_talker + 800.0) / 8 * 128
    assert abs(r["value"] - 128 * 0.08 / (ext / 1e3)) < 1e-9
    # the 1-thread row as bench.py's main asks for it: two runs of 2 frames
    one = bench.cpu_baseline("/m", [1, 2, 3], 1, frames=2, warmup=0, runs=2, target_frames=128)
    assert one is not None and one["cores"] == 1 and len(one["runs"]) == 2


def test_cpu_baseline_one_run_has_no_persistent_lines(monkeypatch, tmp_path):
    """--benchmark-runs 1 prints no [persistent] line in the reference: the
    leg reports a failure (None) instead of a number."""
    exe = tmp_path / "oracle" / "_ref" / "qwen-tts"
    exe.parent.mkdir(parents=True)
    exe.write_text("")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench.subprocess, "run",
                        lambda cmd, **kw: subprocess.CompletedProcess(cmd, 0, "", "Total: 10766.7 ms\n"))
    assert bench.cpu_baseline("/m", [1], 1, frames=2, warmup=0, runs=1) is None
