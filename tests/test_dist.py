"""The N>1 path of bench.py on CPU: world_size-2 gloo ranks agree on the barrier / max / sum and
take disjoint keyspace batches (range split, no collective on the data path)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import bench
    D = bench.Dist()
    D.barrier()
    mx = D.max(float(rank + 1))
    sm = D.sum(float(rank + 1))
    # the batches each rank would walk for 3 steps (bench.bsgs_leg / rmd160_leg partition)
    batches = [s * D.world + D.rank for s in range(3)]
    D.close()
    q.put((rank, mx, sm, batches))


@pytest.mark.parametrize("world", [2])
def test_gloo_barrier_max_and_partition(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    res.sort()
    assert all(r[1] == float(world) for r in res)
    assert all(r[2] == float(world * (world + 1) // 2) for r in res)
    all_batches = [b for r in res for b in r[3]]
    assert sorted(all_batches) == list(range(3 * world))  # disjoint and complete
