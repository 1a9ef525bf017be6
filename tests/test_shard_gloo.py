"""Multi-process (gloo, world_size 2 and 4, CPU) checks of the element-sharded path's
host logic: each rank asks libfks.so which stream words and which elements its shard
owns (fks_shard_census, the same clipping fks_directional_step_shard launches with);
the ranks exchange their census over torch.distributed and check that the shards
tile the stream and write every element of every non-frozen tensor exactly once --
ragged tensors, their tail recomputes and numel < 16 tensors included.  The device
side of the same property is tests/test_gpu_parity.py::test_element_shards_equal_whole."""
import ctypes
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fate_llm.algo.fedkseed import _native as N

SHAPES = [2**18, 37, 3, 2**16 + 16, 185, 624 * 40, 1, 7, 5, 4096 * 3 + 5, 16, 2, 624 * 624 + 9]
FROZEN = {2, 8}


def _arr(shapes):
    arr = (N.FksTensor * len(shapes))()
    for i, n in enumerate(shapes):
        arr[i].data = 4096 * (i + 1)  # aligned fake pointers: the census never dereferences them
        arr[i].numel = n
        arr[i].dtype = N.BF16 if i % 2 else N.F32
        arr[i].flags = N.HAS_WD | (N.FROZEN if i in FROZEN else 0)
    return arr


def census(shard, nshards):
    L = N.load()
    arr = _arr(SHAPES)
    rng = (ctypes.c_int64 * 2)()
    written = (ctypes.c_int64 * len(SHAPES))()
    N.check(L.fks_shard_census(ctypes.addressof(arr), len(SHAPES), shard, nshards, rng, written))
    return (rng[0], rng[1]), list(written)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = census(rank, world)
        everyone = [None] * world
        dist.all_gather_object(everyone, mine)
        # bench.py's timing rule: the job time is the max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((everyone, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_shards_tile_stream_and_write_each_element_once(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    everyone, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world)
    L = N.load()
    arr = _arr(SHAPES)
    words = ctypes.c_int64(0)
    N.check(L.fks_stream_length(ctypes.addressof(arr), len(SHAPES), ctypes.byref(words)))
    ranges = [r for r, _ in everyone]
    assert ranges[0][0] == 0 and ranges[-1][1] >= words.value
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert all(r[1] % 624 == 0 and r[0] % 624 == 0 for r in ranges)
    total = [sum(w[i] for _, w in everyone) for i in range(len(SHAPES))]
    want = [0 if i in FROZEN else n for i, n in enumerate(SHAPES)]
    assert total == want


def test_single_shard_census_is_whole_layout():
    (lo, hi), written = census(0, 1)
    assert lo == 0 and written == [0 if i in FROZEN else n for i, n in enumerate(SHAPES)]
