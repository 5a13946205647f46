"""The N>1 path of bench.py on CPU: world_size-2 gloo ranks agree on the barrier / max / sum, the
partition bench.py actually uses (bench.rank_batch, called by all three legs) gives every rank a
disjoint contiguous run of batches that together cover the keyspace prefix, and `bench.py --gpus N`
started without WORLD_SIZE launches N ranks itself."""
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

from conftest import REPO


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
    # the batches this rank walks for warmup 2 + steps 3, as bsgs_leg / rmd160_leg / xpoint_leg do
    batches = [bench.rank_batch(D.rank, 2, 3, s) for s in range(5)]
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
    assert sorted(all_batches) == list(range(5 * world))  # disjoint and complete


@pytest.mark.parametrize("world", [1, 2, 8])
@pytest.mark.parametrize("warmup,steps", [(0, 1), (2, 10), (5, 20)])
def test_rank_batch_partition(world, warmup, steps):
    import bench
    runs = [[bench.rank_batch(r, warmup, steps, s) for s in range(warmup + steps)] for r in range(world)]
    for run in runs:  # contiguous, so consecutive steps continue the rank's lanes
        assert run == list(range(run[0], run[0] + warmup + steps))
    flat = sorted(b for run in runs for b in run)
    assert flat == list(range(world * (warmup + steps)))  # disjoint and complete, warmup included


def test_bench_gpus_flag_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in p.stderr


def test_bench_launch_ranks_starts_n_processes(tmp_path, capsys):
    """launch_ranks starts N children with RANK/WORLD_SIZE/MASTER_* set and forwards rank 0's stdout
    only; a stand-in child script takes bench.py's place so no GPU is needed."""
    import bench
    script = tmp_path / "child.py"
    script.write_text("import os\nif os.environ['RANK'] == '0':\n"
                      "    print('{\"world\": %s, \"addr\": \"%s\"}' % (os.environ['WORLD_SIZE'], os.environ['MASTER_ADDR']))\n"
                      "raise SystemExit(int(os.environ['RANK']) == 2 and 3)\n")
    rc = bench.launch_ranks(3, [], script=str(script))
    assert rc == 3  # the worst exit status of the ranks
    assert capsys.readouterr().out.strip() == '{"world": 3, "addr": "127.0.0.1"}'
