#!/usr/bin/env python3
"""In-graph spans of the batch-1 frame's kernels from in-kernel stamps
(rocprofv3 durations of graph-replayed dispatches carry a
tracer-widened gap, profiles/r05f_mb_launch_rocprof.txt, so the line also
carries the span the stamps measure).

Runs `bench.py --steps 1 --warmup 0` on the stamp build (lib_s: `make -C
qwen3-tts-c_amd VARIANT=_s EXTRA=-DQTTS_STAMPS`) twice -- QTTS_HIP_GM_DBG=99
(sub-talker pass 5, layer 2: q|k|v GEMV, attention + O, gate|up, down) and
QTTS_HIP_GM_DBG=5 (talker layer 5: q|k|v, O with the merge, gate|up, down) --
parses the `[gm_dbg]` lines of the last frame and writes

  {kernel: {"span_us": first workgroup start -> last stamp,
            "period_us": this launch's first start -> the next stamped launch's,
            "launch_at_us": offset in the stamped group}}

  python tools/graph_spans.py OUT.json
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_S = os.path.join(ROOT, "qwen3-tts-c_amd", "lib_s", "libqwen_tts_amd.so")
# stamped slot -> kernel instantiation (1.7B, batch 1)
NAMES = {"99": {"q|k|v": "k_gemvw<4, 2, false>", "O / -": "k_attn_o<128>", "gate|up": "k_gemvw<6, 2, false>",
                "down": "k_gemvw<1, 6, false>"},
         "5": {"q|k|v": "k_gemvw<4, 4, true>", "O / -": "k_gemvw<2, 4, true, 8>", "gate|up": "k_gemvw<6, 4, true>",
               "down": "k_gemvw<2, 12, true>"}}
PAT = re.compile(r"\[gm_dbg\] (.{8}) launch at\s+([\d.]+) us after the first, last stamp\s+([\d.]+) us into it")


def run(layer):
    env = dict(os.environ, QTTS_LIB=LIB_S, QTTS_HIP_GM_DBG=layer)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                        "--no-profile", "--no-cpu-baseline", "--frames", "16"], env=env, capture_output=True,
                       text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"bench.py (stamp build, GM_DBG={layer}) failed:\n{r.stderr[-2000:]}")
    got = [(m.group(1).strip(), float(m.group(2)), float(m.group(3))) for m in PAT.finditer(r.stderr)]
    got = got[-4:]   # the last frame's group
    out = {}
    for i, (slot, at, span) in enumerate(got):
        nxt = got[i + 1][1] if i + 1 < len(got) else None
        out[NAMES[layer].get(slot, slot)] = {"slot": slot, "span_us": span, "launch_at_us": at,
                                             "period_us": round(nxt - at, 2) if nxt is not None else None,
                                             "group": "sub-talker pass 5 layer 2" if layer == "99" else "talker layer 5"}
    return out, r.stderr


def main():
    res = {}
    logs = []
    for layer in ("99", "5"):
        o, err = run(layer)
        res.update(o)
        logs.append("\n".join(l for l in err.splitlines() if l.startswith("[gm_dbg]")))
    res["_note"] = ("in-kernel s_memrealtime stamps (100 MHz) of one graph-replayed frame on the stamp build; "
                    "span = first workgroup start -> last workgroup's last stamp; period = start -> the next "
                    "stamped launch's start (includes the kernel in between for the talker's O: its attention)")
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1)
    with open(os.path.splitext(sys.argv[1])[0] + ".log", "w") as f:
        f.write("\n\n".join(logs) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
