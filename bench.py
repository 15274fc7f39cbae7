#!/usr/bin/env python3
"""bench.py - Qwen3-TTS hot path on MI355X: audio-seconds per wall-second.

Workload (BASELINE.json metric "audio-sec/wall-sec (RTF^-1) + first-packet ms,
Qwen3-TTS-1.7B @ 1 & 8 GPU"): the 1.7B-shaped synthetic model
(tools/synth_model.py, random init -- no checkpoint offline), the P128 prompt
(SURVEY.md 8d), fixed 128 codec frames per utterance (10.24 s of audio),
default sampling (T 0.9 / top-k 50 / rep 1.05, seed 42), batch 1 per GPU.

One STEP = one full qwen_tts_generate() call through the drop-in C API:
prompt embedding + talker prefill + 128 frames of talker/sub-talker decode
with on-device sampling + codec decode, audio copied back to host memory.

N GPUs (torchrun, one process per GPU): every rank runs its own utterances
(data parallel, no collective in the data path); barrier + synchronize around
the timed region, time = max over ranks, value = total audio seconds / time.

Also reported:
  first_packet_ms  generate() entry -> first 1920 samples available: prefill +
                   frame 0 + codec decode of that frame (the codec is causal,
                   so the first frame decodes on its own; measured after the
                   timed region, on the process's second streaming request:
                   the first also allocates the streaming codec's state and is
                   reported as detail.first_packet_cold_ms)
  roofline         dominant kernel (weight-streaming GEMV), measured live with
                   HIP events on the context stream over one eager frame
  cpu_baseline     the reference c/ build (oracle/_ref/qwen-tts, scalar+OpenMP)
                   on a bounded sample of the same workload, rank 0, N=1 only:
                   3 timed runs of 8 frames at the host cores this process may
                   use, plus a 1-thread row (one 2-frame run), the 128-frame
                   workload extrapolated from the median run
  --eos            the reference's default mode instead of fixed length
                   (max_new_tokens 4096, EOS stop), with the same-length
                   fixed-mode time beside it (eos_mode)
"""
import argparse
import glob
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "qwen3-tts-c_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _pg():
    """True once a torch.distributed process group exists (every multi-rank run;
    a one-rank run with QTTS_BENCH_PG=1, tests/test_dist.py)."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier(ws):
    if ws > 1 or _pg():
        import torch.distributed as dist
        dist.barrier()


def _reduce(ws, v, op):
    if ws == 1 and not _pg():
        return v
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"   # RCCL on the box, gloo in CPU tests
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def reduce_max(ws, v):
    import torch.distributed as dist
    return _reduce(ws, v, dist.ReduceOp.MAX)


def reduce_sum(ws, v):
    import torch.distributed as dist
    return _reduce(ws, v, dist.ReduceOp.SUM)


def rank_prompt_seeds(rank, batch):
    """Utterances of rank r: prompt seeds 1234 + r*batch + i (SURVEY.md 8e:
    independent utterances, static partition, no exchange step)."""
    return [1234 + rank * batch + i for i in range(batch)]


def ensure_model_shared(md, preset, ws, local, overrides=None):
    """local rank 0 of the node writes the model; the others wait."""
    from synth_model import ensure_model
    if local == 0:
        t = time.time()
        ensure_model(md, preset, seed=0, overrides=overrides)
        log(f"[bench] model {preset} ready in {time.time() - t:.1f}s at {md}")
    barrier(ws)


def _latest_profile(pattern):
    """The summary of the profile pass of record: profiles/LATEST names its tag
    (written by tools/gpu_round.sh before the bench line); else the last by name."""
    latest = os.path.join(ROOT, "profiles", "LATEST")
    if os.path.exists(latest):
        tag = open(latest).read().strip()
        fs = glob.glob(os.path.join(ROOT, "profiles", tag + "_" + pattern.lstrip("*")))
        if fs:
            return fs[0]
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    return fs[-1] if fs else None


def _rocprof_lookup(kname, variant=""):
    """Average duration (us) of `kname` in the newest committed rocprofv3
    --stats summary and its HBM bytes per launch in the newest PMC summary
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; tools/prof_summary.py)."""
    avg_us = traffic = None
    src = {}
    f = _latest_profile(f"*{variant}kernel_stats.csv")
    if f:
        import csv
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kname + "(" in row.get("Name", "") or row.get("Name", "").endswith(kname):
                    avg_us = float(row["AverageNs"]) / 1e3
                    src["stats"] = os.path.relpath(f, ROOT)
                    break
    f = _latest_profile(f"*{variant}pmc.json")
    if f:
        with open(f) as fh:
            pm = json.load(fh)
        for name, e in pm.items():
            if kname + "(" in name and "hbm_read_bytes_avg" in e:
                traffic = e["hbm_read_bytes_avg"] + e.get("hbm_write_bytes_avg", 0.0)
                src["pmc"] = os.path.relpath(f, ROOT)
                break
    return avg_us, traffic, src


def profile_roofline(m, lib, variant=""):
    """One eager frame with HIP events around every kernel launch on the
    context stream (qtts_dev_profile_frame); the dominant kernel is the GEMV
    instantiation with the largest share of the frame."""
    import ctypes as C
    n_max = 4096
    kind = (C.c_int * n_max)()
    byt = (C.c_double * n_max)()
    ms = (C.c_float * n_max)()
    names = C.create_string_buffer(n_max * 64)
    lib.qtts_dev_profile_frame.restype = C.c_int
    lib.qtts_dev_profile_frame.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p]
    n = lib.qtts_dev_profile_frame(m.c.hip, 1, n_max, kind, byt, ms, names)
    if n <= 0:
        return None
    k = np.array(kind[:n])
    b = np.array(byt[:n])
    t = np.array(ms[:n], dtype=np.float64)
    nm = [names.raw[i * 64:(i + 1) * 64].split(b"\0", 1)[0].decode() for i in range(n)]
    classes = {0: "gemv_talker", 1: "gemv_subtalker", 2: "attention", 3: "sampler", 4: "embed_sum"}
    share = {classes[i]: float(t[k == i].sum()) for i in classes}
    per_kernel = {}
    for i in range(n):
        e = per_kernel.setdefault(nm[i], [0, 0.0, 0.0])
        e[0] += 1
        e[1] += t[i]
        e[2] += b[i]
    gemv = {x: e for x, e in per_kernel.items() if e[2] > 0}
    dom = max(gemv, key=lambda x: gemv[x][1])
    cnt, tot_ms, tot_b = gemv[dom]
    avg_ms, avg_bytes = tot_ms / cnt, tot_b / cnt
    rp_us, traffic, src = _rocprof_lookup(dom, variant)
    # the in-graph span of the same kernel from in-kernel stamps
    # (tools/graph_spans.py on the stamp build; batch-1 lines only)
    span = None
    f = _latest_profile("*graph_spans.json") if not variant else None
    if f:
        with open(f) as fh:
            e = json.load(fh).get(dom)
        if e:
            span = dict(e, source=os.path.relpath(f, ROOT))
    kind_of = {nm[i]: int(k[i]) for i in range(n)}
    return dict(kernel=dom, kind=kind_of[dom], launches_per_frame=cnt, avg_bytes=avg_bytes, avg_ms=avg_ms,
                achieved_GBs=avg_bytes / (avg_ms * 1e-3) / 1e9, rocprof_avg_us=rp_us, traffic=traffic, in_graph=span,
                profile_src=src, frame_kernel_ms=float(t.sum()), share_ms=share, n_kernels=n,
                kernels={x: {"launches": e[0], "ms": round(e[1], 4), "GBs": round(e[2] / (e[1] * 1e-3) / 1e9, 1)
                             if e[2] else None} for x, e in sorted(per_kernel.items(), key=lambda kv: -kv[1][1])},
                gemv_bytes_per_frame=float(b[(k == 0) | (k == 1)].sum()),
                gemv_ms_per_frame=float(t[(k == 0) | (k == 1)].sum()))


def hbm_stream_bw(lib, gib=2, iters=10):
    """This GPU's own HBM stream bandwidth (the roofline against
    a stream figure measured on the box beside the 8 TB/s nominal):
    qtts_hip_hbm_bw's non-temporal float4 read stream and float4 copy over
    2 GiB buffers (>> the 256 MB Infinity Cache), HIP events on their stream."""
    import ctypes as C
    lib.qtts_hip_hbm_bw.restype = C.c_int
    lib.qtts_hip_hbm_bw.argtypes = [C.c_size_t, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    rd, cp = C.c_double(0), C.c_double(0)
    if lib.qtts_hip_hbm_bw(gib << 30, iters, C.byref(rd), C.byref(cp)) != 0:
        return None
    return {"read_GBs": round(rd.value, 1), "copy_GBs": round(cp.value, 1), "buffer_GiB": gib, "iters": iters,
            "kernel": "qtts_hip_hbm_bw (k_membw.hip): nt float4 loads, 8 per lane in flight, 8 WG x 256 thr per CU"}


def lscpu():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        return {k.strip(): v.strip() for k, v in (l.split(":", 1) for l in out.splitlines() if ":" in l)}
    except Exception:
        return {}


def physical_cores():
    """Physical cores of this host from lscpu (sockets x cores per socket)."""
    try:
        kv = lscpu()
        return int(kv["Socket(s)"]) * int(kv["Core(s) per socket"])
    except Exception:
        return None


def cpu_placement():
    """What the CPU baseline's threads run on: lscpu's SMT width, the CPUs this
    process may use, and the OpenMP placement the reference is started with."""
    kv = lscpu()
    aff = sorted(os.sched_getaffinity(0))
    tpc = kv.get("Thread(s) per core")
    return {"threads_per_core": int(tpc) if tpc and tpc.isdigit() else None,
            "physical_cores": physical_cores(), "affinity_cpus": len(aff),
            "affinity": f"{aff[0]}-{aff[-1]}" if aff and aff[-1] - aff[0] + 1 == len(aff) else ",".join(map(str, aff)),
            "OMP_PLACES": OMP_PLACEMENT["OMP_PLACES"], "OMP_PROC_BIND": OMP_PLACEMENT["OMP_PROC_BIND"]}


# one OpenMP thread per physical core, packed (the reference's GEMV threads
# otherwise float over the share and two can land on one core's SMT pair)
OMP_PLACEMENT = {"OMP_PLACES": "cores", "OMP_PROC_BIND": "close"}
# BASELINE.json configs[1]: greedy decode (the reference CLI's flags for it)
GREEDY_FLAGS = ["--temperature", "1", "--top-k", "1", "--top-p", "1", "--repetition-penalty", "1",
                "--subtalker-temperature", "1", "--subtalker-top-k", "1", "--subtalker-top-p", "1"]
GREEDY = dict(temperature=1.0, top_k=1, top_p=1.0, rep=1.0, st_temperature=1.0, st_top_k=1, st_top_p=1.0)


def cpu_threads_default():
    """Threads for the reference CPU baseline: the physical cores this process
    may use (affinity and OMP_NUM_THREADS bound it: the GPU box gives one GPU's
    job a 16-CPU share and exports OMP_NUM_THREADS=16)."""
    n = len(os.sched_getaffinity(0))
    pc = physical_cores()
    if pc:
        n = min(n, pc)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(md, ids, threads, frames=8, warmup=1, runs=2, target_frames=128, speaker="aiden", timeout=900,
                 greedy=False, wait_policy=None):
    """The reference c/ CLI (oracle/_ref/qwen-tts, built unmodified by
    oracle/Makefile) timed as BASELINE.md §2 plans: --benchmark-warmup /
    --benchmark-runs with the [persistent] lines parsed (c/main.c:262-271).
    The bounded sample decodes `frames` frames per run; the 128-frame
    workload is extrapolated from it: fixed part (prompt + prefill) + talker
    ms/frame x 128 + codec ms/frame x 128 (the reference's decode loop and
    codec are linear in frames)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "qwen-tts")
    if not os.path.exists(exe):
        return None
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), **OMP_PLACEMENT)
    if wait_policy:
        env["OMP_WAIT_POLICY"] = wait_policy
    cmd = [exe, "-d", md, "-t", ",".join(map(str, ids)), "-s", speaker, "-l", "english", "-o", "/tmp/qtts_cpu.wav",
           "--fixed-codec-tokens", str(frames), "--benchmark-warmup", str(warmup), "--benchmark-runs", str(runs), "-v"]
    if greedy:
        cmd += GREEDY_FLAGS
    t = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    wall = time.time() - t
    pr = re.findall(r"\[persistent\] run (\d+)/(\d+): elapsed=([0-9.]+) ms, audio=([0-9.]+)s, talker=([0-9.]+) ms, "
                    r"codec=([0-9.]+) ms, total=([0-9.]+) ms, tokens=(\d+)", r.stderr)
    if r.returncode != 0 or len(pr) != runs:
        log("[bench] cpu baseline failed:", r.stderr[-400:])
        return None
    runs_ = [dict(elapsed_ms=float(p[2]), audio_s=float(p[3]), talker_ms=float(p[4]), codec_ms=float(p[5]),
                  total_ms=float(p[6]), tokens=int(p[7])) for p in pr]
    med = sorted(runs_, key=lambda x: x["total_ms"])[len(runs_) // 2]
    n = med["tokens"]
    fixed_ms = med["total_ms"] - med["talker_ms"] - med["codec_ms"]
    ext_ms = fixed_ms + (med["talker_ms"] + med["codec_ms"]) / n * target_frames
    audio_s = target_frames * 0.08
    return dict(value=audio_s / (ext_ms / 1e3), unit="audio-s/s", cores=threads, kind="reference",
                physical_cores=physical_cores(), placement=dict(cpu_placement(), OMP_WAIT_POLICY=wait_policy),
                runs=runs_,
                sample=(f"reference c/ (oracle/_ref/qwen-tts: unmodified c/ sources, scalar GEMV + OpenMP, no BLAS in "
                        f"the image) on the same synthetic model and prompt{', greedy' if greedy else ''}, {threads} OpenMP "
                        f"threads (OMP_PLACES=cores, OMP_PROC_BIND=close), "
                        f"--fixed-codec-tokens {frames} --benchmark-warmup {warmup} --benchmark-runs {runs} "
                        f"([persistent] lines); the {target_frames}-frame workload is extrapolated from the median run: "
                        f"fixed {fixed_ms:.0f} ms (prompt + prefill) + talker {med['talker_ms'] / n:.0f} ms/frame + codec "
                        f"{med['codec_ms'] / n:.0f} ms/frame -> {ext_ms / 1e3:.1f} s for {audio_s:.2f} s of audio; "
                        f"process wall incl. load {wall:.0f} s"))


def enc_cpu_baseline(md, wav):
    """The voice-clone encoders on the host: the float64 numpy restatement
    (oracle/enc_oracle.py, a port -- the reference's encoders are Python /
    transformers, not runnable here) on ONE reference waveform."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import enc_oracle
    W, scfg, M, mcfg = enc_oracle.load_encoder_weights(md)
    t0 = time.perf_counter()
    enc_oracle.speaker_embedding(W, scfg, wav)
    t1 = time.perf_counter()
    enc_oracle.mimi_encode(M, mcfg, wav)
    t2 = time.perf_counter()
    thr = os.environ.get("OMP_NUM_THREADS") or str(os.cpu_count())
    return dict(speaker_ms=round((t1 - t0) * 1e3, 1), codes_ms=round((t2 - t1) * 1e3, 1), kind="port",
                cores=int(thr), sample=f"oracle/enc_oracle.py (float64 numpy, BLAS threads {thr}) on one "
                                       f"{wav.shape[0] / 24000:.1f} s reference")


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks (one process per
    GPU) through torch.distributed.run as a CHILD process and return its exit
    code.  Runs before anything in this process touches the GPU."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def gather_ranks(ws, rec):
    """Per-rank records {rank, device, utterances, samples, frames, wall_ms} to
    every rank (the only exchange is this gather)."""
    if ws == 1 and not _pg():
        return [rec]
    import torch.distributed as dist
    out = [None] * ws
    dist.all_gather_object(out, rec)
    return out


# bench.py --eos: the codec head's EOS row gain of the synthetic model
# (tools/synth_model.py eos_gain; tools/eos_gain_probe.py: rank 0's P128
# utterance stops at frame 157 under the default sampling at 1.2-1.4)
EOS_GAIN = 1.4

# algorithmic bytes per frame at batch 1 = unique weights +
# talker KV at 2 B/element (bf16) per position
FRAME_WEIGHT_BYTES = {"1.7b": 3.056e9, "0.6b": 1.107e9}
KV_BYTES_PER_POS = 114688


def shared_queue_next(n, step):
    """The cross-GPU work queue's admission hook (qwen_tts_generate_queue's
    `next`): every rank holds the same n utterances and takes the next index
    from one counter in the process group's store (one atomic add per
    utterance, no collective on the data path; `step` = [queue pass] keys a
    fresh counter per pass).  Returns -1 once all n are taken."""
    import torch.distributed as dist
    store = dist.distributed_c10d._get_default_store()

    def nxt():
        i = store.add(f"qtts_queue_{step[0]}", 1) - 1
        return i if i < n else -1
    return nxt


def eos_frames(eos):
    """frames per utterance of an EOS / queue line (None: fixed-length)"""
    if "frames_per_utterance" in eos:
        return eos["frames_per_utterance"]
    if "frames_per_utterance_mean" in eos:
        return eos["frames_per_utterance_mean"]
    q = eos.get("queue")
    return q["frames_per_utterance_mean"] if q else None


def workload_name(args, eos, wavs, vc):
    w = (f"Qwen3-TTS-{args.preset} synthetic, P128 prompt, "
         + (f"fixed {args.frames} frames ({args.frames * 0.08:.2f} s audio), " if not args.eos else "")
         + f"{'greedy' if args.greedy else 'default sampling'}, batch {args.batch} per GPU")
    if args.queue:
        w += (f", work queue of {args.queue} utterances per GPU{' (one shared queue across ranks)' if args.queue_shared else ''}"
              f" through the {args.batch} slots, freed slots refilled inside the live batch")
    if wavs is not None:
        w += (", ICL voice clone from 5 s reference audio (12 Hz codes + x-vector encoded on the GPU inside the "
              "step) + 20-id reference text, codec over reference ++ generated (reference part cut)")
    elif vc:
        w += (", ICL voice clone: 63 reference frames + 20-id reference text + x-vector, codec over reference ++ "
              "generated (reference part cut)")
    elif args.eos:
        f = eos_frames(eos) if eos else None
        w += (f", EOS mode (max_new_tokens 4096, codec-head EOS row x {EOS_GAIN}: the utterances stop at frame {f}"
              f"{'' if 'frames_per_utterance' in (eos or {}) else ' on average'})")
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--preset", default="1.7b")
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--greedy", action="store_true",
                    help="greedy decode (top-k 1, temperature 1, no repetition penalty; BASELINE.json configs[1] "
                         "with --preset 0.6b)")
    ap.add_argument("--batch", type=int, default=1, help="utterances per GPU per step (lock-step batch)")
    ap.add_argument("--cpu-frames", type=int, default=8, help="frames per run of the bounded CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the physical cores this process may use")
    ap.add_argument("--cpu-runs", type=int, default=3, help="timed runs of the CPU-baseline sample (SURVEY.md 8d: 3)")
    ap.add_argument("--no-cpu-1thread", action="store_true", help="skip the reference's 1-thread row")
    ap.add_argument("--cpu-1thread", action="store_true", help="(C1 line) also time the reference with 1 thread")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--model-dir", default=None)
    ap.add_argument("--voice-clone", action="store_true",
                    help="BASELINE C5: ICL voice clone from 5 s of synthetic reference AUDIO per utterance "
                         "(12 Hz encoder + speaker encoder on the GPU, inside the timed step) + reference text, "
                         "decode of reference ++ generated")
    ap.add_argument("--vc-codes", action="store_true",
                    help="with --voice-clone: start from seeded reference codes + x-vector (no audio encode)")
    ap.add_argument("--eos", action="store_true",
                    help="the reference's default generation mode: max_new_tokens 4096 with the EOS stop, on the "
                         "synthetic model with the codec head's EOS row x EOS_GAIN (its utterance stops at frame 157); "
                         "also times fixed-length decodes of the same length")
    ap.add_argument("--queue", type=int, default=0,
                    help="work queue (SURVEY.md 8(e)): this many utterances per GPU per step through --batch "
                         "lock-step slots, each freed slot refilled inside the live batch (qwen_tts_generate_queue); "
                         "with --eos the utterances stop at their own EOS")
    ap.add_argument("--queue-shared", action="store_true",
                    help="with --queue: one queue of queue x gpus utterances for all ranks, each rank admitting the "
                         "next index from a counter in the process group's store (a dynamic cross-GPU work queue, "
                         "no collective in the data path)")
    ap.add_argument("--c1", action="store_true",
                    help="BASELINE C1 only: the reference c/ CLI on the 0.6B synthetic model, short prompt "
                         "(test/tokens_great_power.txt), on the host cores; no GPU")
    args = ap.parse_args()

    if args.c1:
        return c1_line(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))

    ws, rank, local = dist_setup()
    if ws != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    import torch
    # one process per GPU; QTTS_BENCH_BACKEND=gloo rehearses N ranks on fewer
    # GPUs (ranks share devices round-robin), RCCL ("nccl") otherwise
    backend = os.environ.get("QTTS_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev = local % ndev if ndev else local
    if ws > 1 or os.environ.get("QTTS_BENCH_PG") == "1":
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        log(f"[bench] rank {rank}: process group {dist.get_backend()} (world {dist.get_world_size()}, device {dev})")
    import qtts
    from synth_model import prompt_ids

    # the same synthetic dir the GPU tests generate (tests/conftest.py model_dir): one 3.4 GB write per box
    ovr = {"eos_gain": EOS_GAIN} if args.eos else None
    mtag = args.preset + (f"_eos_gain{EOS_GAIN}" if args.eos else "")
    md = args.model_dir or os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), mtag)
    ensure_model_shared(md, args.preset, ws, local, ovr)
    t = time.time()
    m = qtts.QwenTTS(md, device=dev)
    log(f"[bench] rank {rank}: model loaded on HIP device {dev} in {time.time() - t:.1f}s")
    samp = GREEDY if args.greedy else {}
    if args.eos:   # the reference's defaults: max_new_tokens 4096, EOS stop (Q.c:871-880, 1324-1330)
        m.set_params(max_tokens=4096, fixed=0, seed=42 + rank, **samp)
    else:
        m.set_params(max_tokens=args.frames, fixed=args.frames, seed=42 + rank, **samp)
    prompts = [prompt_ids("p128", seed=sd) for sd in rank_prompt_seeds(rank, args.batch)]
    qprompts, qnext, qstep = None, None, [0]
    if args.queue:
        if args.queue_shared:   # every rank holds the whole list; a store counter hands out indices
            qprompts = [prompt_ids("p128", seed=1234 + i) for i in range(args.queue * ws)]
            if ws > 1:
                qnext = shared_queue_next(len(qprompts), qstep)
        else:
            qprompts = [prompt_ids("p128", seed=sd) for sd in rank_prompt_seeds(rank, args.queue)]
    qstats = []
    last_audio = [None]

    vc = None
    wavs = None
    if args.voice_clone:
        # 5 s of reference audio (63 frames at 12.5 Hz); reference
        # text = chat template around 20 seeded ids.  Default: the audio itself,
        # encoded on the GPU inside the step; --vc-codes: seeded codes + x-vector
        import numpy as np
        from synth_model import ref_wave
        H = m.cfg.talker_hidden
        vc = []
        wavs = []
        for i, sd in enumerate(rank_prompt_seeds(rank, args.batch)):
            r = np.random.default_rng(sd + 7)
            codes = r.integers(0, 2048, size=(63, m.cfg.num_code_groups)).astype(np.int32)
            rids = [151644, 77091, 198] + r.integers(1000, 100000, size=20).tolist() + [151645, 198]
            vc.append((rids, codes, (r.standard_normal(H) * 0.05).astype(np.float32)))
            wavs.append(ref_wave(sd + 7, 5.0))
        if args.vc_codes:
            wavs = None
        elif m.encoders_available() != 3:
            raise SystemExit("bench.py --voice-clone: the model dir has no audio encoders (use --vc-codes)")

    def one_step():
        if wavs is not None:
            rc, aud = m.generate_voice_clone_audio_batch(prompts, wavs, [v[0] for v in vc],
                                                         ["english"] * args.batch)
            if rc != 0:
                raise RuntimeError("voice-clone (reference audio) generation failed")
            return sum(len(a) for a in aud)
        if vc is not None:
            rc, aud = m.generate_voice_clone_batch(prompts, [v[0] for v in vc], [v[1] for v in vc],
                                                   [v[2] for v in vc], ["english"] * args.batch)
            if rc != 0:
                raise RuntimeError("voice-clone generation failed")
            return sum(len(a) for a in aud)
        if qprompts is not None:
            n = len(qprompts)
            rc, aud = m.generate_queue(qprompts, ["aiden"] * n, ["english"] * n, slots=args.batch, next_fn=qnext)
            qstep[0] += 1
            if rc != 0:
                raise RuntimeError("queue generation failed")
            qstats.append(m.queue_stats())
            return sum(len(a) for a in aud if a is not None)
        if args.batch == 1:
            a = m.generate(prompts[0], "aiden", "english")
            if a is None:
                raise RuntimeError("generation produced no audio")
            return len(a)
        rc, aud = m.generate_batch(prompts, ["aiden"] * args.batch, ["english"] * args.batch)
        if rc != 0:
            raise RuntimeError("batch generation failed")
        last_audio[0] = aud
        return sum(len(a) for a in aud)

    for _ in range(args.warmup):
        one_step()
    qstats.clear()
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = 0
    for _ in range(args.steps):
        samples += one_step()
    torch.cuda.synchronize()
    barrier(ws)
    el = time.perf_counter() - t0
    # the last timed step's phases (run_batch's perf_* fields: prefill, decode
    # loop, codec -- for a batch, every slot's codec pass)
    phases = dict(prefill_ms=m.c.perf_prefill_ms, talker_ms=m.c.perf_talker_ms, codec_ms=m.c.perf_codec_ms)
    eos = None
    if args.eos:
        # the same utterances at the same length in fixed-length mode: what the
        # EOS mode itself costs (host polling every 8 frames, the attention grid
        # sized from the 4096-frame KV capacity)
        # (batch 1 only: the slots of a batch stop at different frames, so one
        # fixed length would be a different workload; there the line reports
        # the mean frames per utterance alone)
        if args.batch == 1 and not args.queue:
            n_eos = samples // (1920 * args.steps)
            m.set_params(max_tokens=n_eos, fixed=n_eos, seed=42 + rank, **samp)
            one_step()
            torch.cuda.synchronize()
            tf = time.perf_counter()
            sf = sum(one_step() for _ in range(args.steps))
            torch.cuda.synchronize()
            elf = time.perf_counter() - tf
            m.set_params(max_tokens=4096, fixed=0, seed=42 + rank, **samp)
            eos = dict(eos_gain=EOS_GAIN, frames_per_utterance=n_eos, max_new_tokens=4096,
                       fixed_same_length_audio_s_per_s=round(sf / 24000.0 / elf, 3),
                       fixed_same_length_ms_per_step=round(elf / args.steps * 1e3, 2))
        elif not args.queue:
            eos = dict(eos_gain=EOS_GAIN, frames_per_utterance_mean=round(samples / (1920 * args.steps * args.batch), 2),
                       max_new_tokens=4096)
            # a lock-step batch runs every slot to the longest one (+ the one
            # frame of the lagged stop poll): useful slot-frames / launched
            fr = [len(a) // 1920 for a in last_audio[0]] if last_audio[0] else []
            if fr:
                eos["slot_occupancy"] = round(sum(fr) / (args.batch * (max(fr) + 1)), 4)
                eos["frames_per_slot_last_step"] = fr
        else:
            eos = dict(eos_gain=EOS_GAIN, max_new_tokens=4096)
    if qstats:
        used = sum(q["used"] for q in qstats)
        launched = sum(q["frames"] for q in qstats)
        rows = sum(q["rows_launched"] for q in qstats)
        nq_done = sum(sum(1 for f in q["frames_per_utt"] if f >= 0) for q in qstats)
        qd = dict(utterances_per_step=args.queue * (ws if args.queue_shared else 1), slots=args.batch,
                  shared_across_ranks=bool(args.queue_shared),
                  utterances_this_rank=nq_done, refills=sum(q["refills"] for q in qstats),
                  frames_launched=launched, useful_slot_frames=used,
                  rows_launched=rows,
                  slot_occupancy=round(used / rows, 4) if rows else None,
                  slot_occupancy_full_width=round(used / (args.batch * launched), 4) if launched else None,
                  occupancy_note="useful slot-frames / slot rows launched (the tail, with nothing left to admit, "
                                 "moves the running utterances to the first slots and launches those rows only); "
                                 "full_width: / (slots x frames launched)",
                  useful_frames_per_s=round(used / el, 1),
                  frames_per_utterance_mean=round(used / max(nq_done, 1), 2),
                  lock_step_occupancy_same_utterances=None)
        # the same utterances as lock-step batches of `slots` (in queue order):
        # each batch runs to its longest utterance + the lagged poll's frame
        q = qstats[-1]
        fr = [f for f in q["frames_per_utt"] if f > 0]
        if fr and not args.queue_shared:
            ls = sum(max(fr[i:i + args.batch]) + 1 for i in range(0, len(fr), args.batch))
            qd["lock_step_occupancy_same_utterances"] = round(sum(fr) / (args.batch * ls), 4)
        if eos is not None:
            eos.update(queue=qd)
        else:
            eos = dict(queue=qd)
    el_max = reduce_max(ws, el)
    audio_total = reduce_sum(ws, samples / 24000.0)
    value = audio_total / el_max
    ms_per_step = el_max / args.steps * 1e3
    n_utt = (sum(sum(1 for f in q["frames_per_utt"] if f >= 0) for q in qstats) if qstats
             else args.batch * args.steps)
    ranks = gather_ranks(ws, dict(rank=rank, device=dev, utterances=n_utt, samples=samples,
                                  frames=samples // 1920, wall_ms=round(el * 1e3, 2)))

    # ---- first packet (BASELINE.json metric, configs[2]): streaming generation,
    # wall time from the call to the first audio chunk (frame 0 decoded by the
    # exact streaming codec and on the host) ----
    fp = None
    if args.batch == 1 and vc is None:
        m.generate(prompts[0], "aiden", "english")       # non-streaming breakdown
        prefill_ms, talker_ms, codec_ms = m.c.perf_prefill_ms, m.c.perf_talker_ms, m.c.perf_codec_ms
        # the first streaming request of the process also allocates the
        # streaming codec's state (reported as first_packet_cold_ms); the line
        # reports the second request, as a serving process sees it
        first = []
        m.generate_stream(prompts[0], "aiden", "english", chunk_frames=8, on_chunk=first.append)
        cold_ms = m.c.perf_first_packet_ms
        first = []
        m.generate_stream(prompts[0], "aiden", "english", chunk_frames=8, on_chunk=first.append)
        fp = dict(first_packet_ms=m.c.perf_first_packet_ms, first_packet_cold_ms=cold_ms,
                  first_frame_ms=m.c.perf_first_frame_ms,
                  first_packet_samples=int(len(first[0])) if first else 0, stream_chunk_frames=8,
                  prefill_ms=prefill_ms, talker_ms=talker_ms, codec_ms=codec_ms)

    enc = None
    if wavs is not None:
        # the reference-audio encode of one step alone (both encoders, whole batch)
        m.speaker_embed(wavs)
        m.encode_audio(wavs)
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(3):
            m.speaker_embed(wavs)
        ts = time.perf_counter()
        for _ in range(3):
            m.encode_audio(wavs)
        tc = time.perf_counter()
        gf = encoder_gflop(md, [w.shape[0] for w in wavs])
        spk_ms, cod_ms = (ts - te) / 3 * 1e3, (tc - ts) / 3 * 1e3
        enc = dict(speaker_ms=round(spk_ms, 3), codes_ms=round(cod_ms, 3), ref_seconds=5.0, batch=len(wavs),
                   cpu_baseline=None if (args.no_cpu_baseline or rank != 0) else enc_cpu_baseline(md, wavs[0]),
                   speaker_gflop=round(gf[0], 2), codes_gflop=round(gf[1], 2),
                   speaker_tflops=round(gf[0] / spk_ms, 2), codes_tflops=round(gf[1] / cod_ms, 2),
                   note="wall time of the encoder call (host waveform in, host codes / x-vectors out), "
                        "dense-contraction GFLOP counted per SURVEY.md 8f N3 shapes")
    if args.batch == 1 and vc is not None:
        # voice-clone first packet: reference frames through the streaming codec, then frame 0
        for _ in range(2):   # second request, as for the custom-voice line
            m.generate_voice_clone_stream(prompts[0], vc[0][0], vc[0][1], vc[0][2], "english", chunk_frames=8)
        fp = dict(first_packet_ms=m.c.perf_first_packet_ms, first_frame_ms=m.c.perf_first_frame_ms,
                  prefill_ms=m.c.perf_prefill_ms, ref_frames=63)
        if wavs is not None:
            # the same from the 5 s reference AUDIO: the encode is on the first-packet path
            for _ in range(2):
                m.generate_voice_clone_audio_stream(prompts[0], wavs[0], vc[0][0], "english", chunk_frames=8)
            fp["first_packet_from_audio_ms"] = m.c.perf_first_packet_ms
    # (the 0.6B line reads the 0.6B profile passes: <tag>_06b_kernel_stats.csv / _pmc.json;
    # a batch-B line its own: <tag>_b8_kernel_stats.csv / _b8_pmc.json)
    # (a voice-clone line reads its own passes: <tag>_vc8_kernel_stats.csv / _vc8_pmc.json)
    pvar = ("" if args.preset == "1.7b" else args.preset.replace(".", "") + "_") + \
        (f"vc{args.batch}_" if vc is not None else f"b{args.batch}_" if args.batch > 1 else "")
    roof = None if args.no_profile else profile_roofline(m, qtts.lib(), pvar)
    hbm = None if args.no_profile else hbm_stream_bw(qtts.lib())
    m.close()

    cpu = None
    # the reference c/ CPU leg belongs to the custom-voice line (the c/ reference
    # has no voice clone); a voice-clone line carries the encoders' host port
    # baseline in ref_audio_encode instead
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and vc is None and not args.eos:
        thr = args.cpu_threads or cpu_threads_default()
        cpu = cpu_baseline(md, prompts[0], thr, frames=args.cpu_frames, runs=args.cpu_runs, target_frames=args.frames,
                           greedy=args.greedy)
        if cpu and not args.no_cpu_1thread:
            # (two measured runs: the reference prints its [persistent] lines only
            # for --benchmark-runs > 1, c/main.c:263-264)
            one = cpu_baseline(md, prompts[0], 1, frames=2, warmup=0, runs=2, target_frames=args.frames, timeout=3000,
                               greedy=args.greedy)
            if one:
                cpu["one_thread"] = {k: one[k] for k in ("value", "unit", "cores", "sample", "runs")}

    if rank == 0:
        out = {
            "metric": "audio-sec/wall-sec (RTF^-1) + first-packet ms, Qwen3-TTS-1.7B @ 1 & 8 GPU",
            "value": round(value, 3),
            "unit": "audio-s/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32 activations x bf16 weights (fp32 accumulate)",
            "data": f"synthetic (seeded random-init weights of the {args.preset.upper()} architecture, tools/synth_model.py)",
            "config": {"workload": workload_name(args, eos, wavs, vc),
                       "global_batch": (args.queue * ws if args.queue else args.batch * ws),
                       "frames": eos_frames(eos) if eos and eos_frames(eos) is not None else args.frames,
                       "parallelism": f"dp{ws} (independent replicas, no collective in the data path"
                                      + ("; utterance indices from a shared store counter" if args.queue_shared else "")
                                      + ")"},
        }
        if fp:
            out["first_packet_ms"] = round(fp["first_packet_ms"], 2)
        # batch 1: the first-packet request's fields, then the last timed step's
        # phases as step_*; a batch: the phases
        det = dict(fp, **{"step_" + k: v for k, v in phases.items()}) if fp else phases
        out["detail"] = {k: round(v, 2) if isinstance(v, float) else v for k, v in det.items()}
        out["ranks"] = ranks
        if enc:
            out["ref_audio_encode"] = enc
        if eos:
            out["eos_mode"] = eos
        fw = FRAME_WEIGHT_BYTES.get(args.preset)
        if fw and vc is None and not args.eos:
            # §8(d) headline: utterance-frames per second x algorithmic bytes per
            # frame (weights once per lock-step step + B x KV) over 8 TB/s; the
            # mean talker position is prefill (10 rows: 3 role + 7 codec-prefix
            # rows, speaker and language set) + the frames before it
            pos = 10 + (args.frames - 1) / 2.0
            fps = value / 0.08                                  # 12.5 frames per audio second
            steps_ps = fps / args.batch
            ach = (steps_ps * fw + fps * KV_BYTES_PER_POS * pos) / 1e9
            ach32 = (steps_ps * fw + fps * 2 * KV_BYTES_PER_POS * pos) / 1e9
            out["roofline_frame"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(ach / HBM_PEAK_GBS, 4), "frames_per_s": round(fps, 1),
                                     "bytes_per_frame": int(fw + KV_BYTES_PER_POS * pos * args.batch) // args.batch,
                                     "mean_kv_pos": pos,
                                     "achieved_fp32_kv": round(ach32, 1),
                                     "measured_stream": hbm,
                                     "frac_of_measured_read": round(ach / hbm["read_GBs"], 4) if hbm else None,
                                     "note": "SURVEY.md 8(d): frames/s x (W + 114688 B x pos) / 8 TB/s, KV at 2 B/elem; "
                                             "this build keeps the reference's fp32 KV (achieved_fp32_kv counts it); "
                                             "whole utterance wall (prefill + codec included)"}
        if roof:
            # sub-talker kernels (GEMVs, attention + O) read weights the Infinity
            # Cache holds (224 MB, 16 reads per frame) and are latency-bound
            bound = "mall/latency" if roof["kind"] in (1, 2) else "hbm"
            out["roofline"] = {"bound": bound, "achieved": round(roof["achieved_GBs"], 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(roof["achieved_GBs"] / HBM_PEAK_GBS, 4),
                               "traffic": None if roof["traffic"] is None else int(roof["traffic"]),
                               "kernel": roof["kernel"],
                               "avg_launch_us": round(roof["avg_ms"] * 1e3, 2),
                               "rocprof_avg_us": None if roof["rocprof_avg_us"] is None
                               else round(roof["rocprof_avg_us"], 2),
                               "avg_launch_bytes": int(roof["avg_bytes"]),
                               "in_graph_span_us": roof["in_graph"]["span_us"] if roof.get("in_graph") else None,
                               "in_graph_period_us": roof["in_graph"]["period_us"] if roof.get("in_graph") else None,
                               "frac_in_graph_span": round(roof["avg_bytes"] / (roof["in_graph"]["span_us"] * 1e-6) / 1e9
                                                           / HBM_PEAK_GBS, 4) if roof.get("in_graph") else None,
                               "in_graph_source": roof["in_graph"]["source"] if roof.get("in_graph") else None,
                               "launches_per_frame": roof["launches_per_frame"],
                               "measured_stream": hbm,
                               "frac_of_measured_read": round(roof["achieved_GBs"] / hbm["read_GBs"], 4) if hbm else None,
                               "profiles": roof["profile_src"]}
            out["frame_profile"] = {"kernel_ms_per_frame": round(roof["frame_kernel_ms"], 3),
                                    "share_ms": {k: round(v, 3) for k, v in roof["share_ms"].items()},
                                    "gemv_GBs_all": round(roof["gemv_bytes_per_frame"] /
                                                          (roof["gemv_ms_per_frame"] * 1e-3) / 1e9, 1),
                                    "kernels": roof["kernels"],
                                    "n_kernels": roof["n_kernels"]}
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def encoder_gflop(md, lens):
    """Dense-contraction GFLOP of the voice-clone encoders (2 flop per MAC) for
    reference waveforms of `lens` samples: (speaker encoder incl. the STFT,
    12 Hz encoder incl. the codebook distances)."""
    cfg = json.load(open(os.path.join(md, "config.json"))).get("speaker_encoder_config", {})
    mc = json.load(open(os.path.join(md, "speech_tokenizer", "config.json"))).get("encoder_config", {})
    ch, ks = cfg.get("enc_channels", [512, 512, 512, 512, 1536]), cfg.get("enc_kernel_sizes", [5, 3, 3, 3, 1])
    sc, att, se = cfg.get("enc_res2net_scale", 8), cfg.get("enc_attention_channels", 128), cfg.get("enc_se_channels", 128)
    spk = cod = 0.0
    for n in lens:
        T = (n - 256) // 256 + 1
        macs = 1026 * 1024 * T + 128 * 513 * T                        # STFT basis + mel
        macs += ch[0] * 128 * ks[0] * T
        for i in range(1, len(ch) - 1):
            macs += 2 * ch[i] * ch[i - 1] * T + (sc - 1) * (ch[i] // sc) ** 2 * ks[i] * T + 2 * se * ch[i]
        macs += ch[-1] * ch[-1] * T + att * 3 * ch[-1] * T + ch[-1] * att * T + 2 * ch[-1] * cfg.get("enc_dim", 2048)
        spk += 2 * macs
        nf, hid = mc.get("num_filters", 64), mc.get("hidden_size", 512)
        L, C = n, nf
        macs = nf * 7 * L
        for r in reversed(mc.get("upsampling_ratios", [8, 6, 5, 4])):
            macs += (C // 2) * C * 3 * L + C * (C // 2) * L
            L = -(-L // r)
            macs += 2 * C * C * 2 * r * L
            C *= 2
        macs += hid * C * 3 * L
        I = mc.get("intermediate_size", 2048)
        qd = mc.get("num_attention_heads", 8) * mc.get("head_dim", 64)
        w = min(L, mc.get("sliding_window", 250))
        macs += mc.get("num_hidden_layers", 8) * L * (4 * hid * qd + 2 * hid * I + 2 * qd * w)
        T12 = -(-L // 2)
        vq = mc.get("vector_quantization_hidden_dimension", 256)
        macs += hid * hid * 4 * T12 + 2 * vq * hid * T12 + 16 * T12 * mc.get("codebook_size", 2048) * vq
        cod += 2 * macs
    return spk / 1e9, cod / 1e9


def c1_line(args):
    """BASELINE C1: 0.6B, single short prompt, the reference c/ BLAS+OpenMP
    path (here: scalar + OpenMP, no BLAS in the image), host cores only."""
    from synth_model import ensure_model, prompt_ids
    md = args.model_dir or os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "0.6b")
    ensure_model(md, "0.6b", seed=0)
    thr = args.cpu_threads or cpu_threads_default()
    rows = {}
    for t in ([thr, 1] if args.cpu_1thread else [thr]):
        fr = args.cpu_frames if t > 1 else 2   # the 1-thread row: a 2-frame sample
        r = cpu_baseline(md, prompt_ids("short"), t, frames=fr, warmup=1 if t > 1 else 0, runs=2,
                         target_frames=args.cpu_frames, timeout=3000)
        rows[str(t)] = r
    out = {"metric": "audio-sec/wall-sec (RTF^-1), reference c/ CPU path (BASELINE C1)", "unit": "audio-s/s",
           "value": rows[str(thr)]["value"] if rows.get(str(thr)) else None, "higher_is_better": True,
           "config": {"workload": f"Qwen3-TTS-0.6b synthetic, short prompt (test/tokens_great_power.txt), "
                                  f"fixed {args.cpu_frames} frames, default sampling"},
           "data": "synthetic (seeded random-init weights of the 0.6B architecture, tools/synth_model.py)",
           "rows": rows}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
