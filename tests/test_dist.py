"""The multi-GPU path on CPU: bench.py's partition and reductions under a
world_size-2 gloo group (the box runs the same code over RCCL).  Utterances
are independent: ranks get disjoint prompts, no data-path
collective exists, and the reported value is sum(audio) / max(wall)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    w, r, local = bench.dist_setup()
    seeds = bench.rank_prompt_seeds(r, 3)
    el = bench.reduce_max(w, 1.0 + r)            # per-rank wall time
    audio = bench.reduce_sum(w, 10.24 * (r + 1))  # per-rank audio seconds
    bench.barrier(w)
    q.put((r, w, local, seeds, el, audio))
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2])
def test_partition_and_reductions_gloo(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_seeds = [s for r in res for s in r[3]]
    assert len(set(all_seeds)) == len(all_seeds) == 3 * ws       # disjoint utterances
    for r, w, local, seeds, el, audio in res:
        assert w == ws and local == r
        assert el == pytest.approx(float(ws))                      # max over ranks
        assert audio == pytest.approx(10.24 * ws * (ws + 1) / 2)   # sum over ranks


def test_single_rank_is_identity():
    assert bench.reduce_max(1, 3.5) == 3.5 and bench.reduce_sum(1, 2.0) == 2.0
    assert bench.rank_prompt_seeds(0, 2) == [1234, 1235]


def _gen_worker(rank, ws, port, tiny_dir, q):
    """One rank of the data-parallel bench on CPU: its own prompts (bench's
    static partition), decoded by the oracle (the CPU checker stands in for
    the HIP path, which needs the GPU), then bench's per-rank gather."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from oracle_py import Oracle, GREEDY
    from qtts_io import lookup_ids
    from synth_model import prompt_ids
    w, r, _ = bench.dist_setup()
    o = Oracle(tiny_dir)
    s, l = lookup_ids(o.cfg, "aiden", "english")
    codes = []
    for sd in bench.rank_prompt_seeds(r, 2):
        c, _ = o.generate_codes(prompt_ids("p128", seed=sd), s, l, max_tokens=4096, fixed=2, seed=42, **GREEDY)
        codes.append(c.tolist())
    o.close()
    recs = bench.gather_ranks(w, dict(rank=r, samples=2 * 2 * 1920, frames=4, wall_ms=10.0 * (r + 1), codes=codes))
    q.put((r, recs))
    dist.destroy_process_group()


def test_two_rank_generate_gather_gloo(tiny_dir):
    """world_size 2 on gloo: each rank decodes its own utterances, bench's
    gather gives every rank every record, and each rank's codes equal a
    single-process decode of the same prompts (ranks share nothing)."""
    from oracle_py import Oracle, GREEDY
    from qtts_io import lookup_ids
    from synth_model import prompt_ids
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gen_worker, args=(r, ws, port, tiny_dir, q)) for r in range(ws)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(ws))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] and [x["rank"] for x in res[0]] == [0, 1]
    o = Oracle(tiny_dir)
    s, l = lookup_ids(o.cfg, "aiden", "english")
    for rec in res[0]:
        for sd, got in zip(bench.rank_prompt_seeds(rec["rank"], 2), rec["codes"]):
            want, _ = o.generate_codes(prompt_ids("p128", seed=sd), s, l, max_tokens=4096, fixed=2, seed=42, **GREEDY)
            assert got == want.tolist()
    o.close()


def _queue_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    import time
    step = [0]
    got = {}
    for p in range(2):                       # two queue passes: a fresh counter each
        nxt = bench.shared_queue_next(13, step)
        mine = []
        while True:
            i = nxt()
            if i < 0:
                break
            mine.append(i)
            time.sleep(0.002 * (rank + 1))   # uneven per-utterance cost
        got[p] = mine
        step[0] += 1
        bench.barrier(ws)
    q.put((rank, got))
    dist.destroy_process_group()


def test_shared_queue_counter_gloo():
    """bench.py --queue-shared on world_size 2 gloo: ranks admit utterance
    indices from one store counter (qwen_tts_generate_queue's `next` hook);
    every index of every pass is taken exactly once, by whichever rank asks
    first -- the slower rank takes fewer."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_queue_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(ws))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for pss in range(2):
        taken = res[0][pss] + res[1][pss]
        assert sorted(taken) == list(range(13)), (pss, res)
        assert res[0][pss] and res[1][pss]


@pytest.mark.gpu
def test_bench_shared_queue_two_ranks(gpu):
    """`bench.py --gpus 2 --queue 5 --queue-shared --batch 2 --eos` on one box
    (two ranks sharing the GPU over gloo): the two ranks' queues drain ONE list
    of 10 EOS-mode utterances between them; every utterance is decoded once."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QTTS_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--preset", "tiny", "--eos",
                        "--batch", "2", "--queue", "5", "--queue-shared", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--no-profile"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    qd = line["eos_mode"]["queue"]
    assert qd["shared_across_ranks"] and qd["utterances_per_step"] == 10
    assert line["config"]["global_batch"] == 10
    assert sum(x["utterances"] for x in line["ranks"]) == 10, line["ranks"]


@pytest.mark.gpu
def test_bench_gpus2_self_launch(gpu):
    """`bench.py --gpus 2` starts its own 2 ranks (no external launcher); on a
    one-GPU box both share it over gloo.  The line reports n_gpus 2 and one
    record per rank."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QTTS_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--preset", "tiny",
                        "--frames", "4", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-profile"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2
    assert sorted(x["rank"] for x in line["ranks"]) == [0, 1]
    assert all(x["samples"] == 4 * 1920 for x in line["ranks"])


@pytest.mark.gpu
def test_bench_rccl_process_group_one_rank(gpu):
    """bench.py under torch.distributed.run with an RCCL ("nccl") process group
    of one rank on cuda:0 (QTTS_BENCH_PG=1): the init with device_id, the
    barriers around the timed region, the max / sum all-reduces on CUDA tensors
    and the all_gather_object of the rank records all run through RCCL -- the
    code the driver's 8-GPU scaling run takes, on the one GPU this box has."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QTTS_BENCH_PG="1")
    env.pop("QTTS_BENCH_BACKEND", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
                        os.path.join(root, "bench.py"), "--gpus", "1", "--preset", "tiny", "--frames", "4",
                        "--steps", "2", "--warmup", "0", "--no-cpu-baseline", "--no-profile"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "process group nccl (world 1, device 0)" in r.stderr, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1 and [x["rank"] for x in line["ranks"]] == [0]
    assert line["ranks"][0]["samples"] == 2 * 4 * 1920 and line["value"] > 0
