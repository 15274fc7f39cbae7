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
