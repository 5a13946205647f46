"""The N>1 path of bench.py on CPU: world_size-2 gloo ranks agree on the barrier / max / sum / gather,
the partition bench.py actually uses (bench.rank_origin, called by all three legs) gives every rank a
disjoint contiguous region, the step batch is sized for the sustained window, more ranks than GPUs
is refused unless --rehearse, and `bench.py --gpus N` started without WORLD_SIZE launches N ranks
itself."""
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
    # the region this rank walks (bsgs_leg / address_leg): units [origin, origin + span)
    origin = bench.rank_origin(D.rank, bench.RANK_SPAN_BASES)
    got = D.gather({"rank": D.rank, "origin": origin})
    D.close()
    q.put((rank, mx, sm, origin, got))


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
    origins = [r[3] for r in res]
    assert origins == [r * (1 << 40) for r in range(world)]
    assert all(r[4] == [{"rank": i, "origin": origins[i]} for i in range(world)] for r in res)  # gather, rank order


@pytest.mark.parametrize("world", [1, 2, 8])
def test_rank_regions_disjoint_and_inside_the_range(world):
    """Rank regions [origin, origin + span) of BSGS bases and 2^32-key chunks never overlap, and the
    8-rank job stays inside each workload's -b range and short of its puzzle key (the legs assert
    that nothing is found while timing)."""
    import bench
    for span, unit_keys, lo, key in ((bench.RANK_SPAN_BASES, 2 << 44, 1 << 124, 0x1c533b6bb7f0804e09960225e44877ac),
                                     (bench.RANK_SPAN_BASES, 2 << 44, 1 << 129, 0x33e7665705359f04f28b88cf897c603c9),
                                     (bench.RANK_SPAN_CHUNKS, 1 << 32, 1 << 65, 0x2832ed74f2b5e35ee),
                                     (bench.RANK_SPAN_CHUNKS, 1 << 32, 1 << 62, 0x7cce5efdaccf6808)):
        regions = sorted((bench.rank_origin(r, span), bench.rank_origin(r, span) + span) for r in range(world))
        assert all(a[1] <= b[0] for a, b in zip(regions, regions[1:]))
        assert lo + regions[-1][1] * unit_keys <= key < 2 * lo


@pytest.mark.parametrize("walks", [1, 2, 4])
def test_walk_parts_tile_the_rank_region(walks):
    """bench.py --walks S cuts each rank region into S contiguous parts, one per context: the parts
    are disjoint, lie inside the rank's region and, walked as far as the part allows, end at the next
    part's start."""
    import bench
    for span, unit_keys in ((bench.RANK_SPAN_BASES, 2 << 44), (bench.RANK_SPAN_CHUNKS, 1 << 32)):
        for rank in range(8):
            origin = (1 << 124) + bench.rank_origin(rank, span) * unit_keys
            starts = [bench.walk_origin(origin, i, walks, span, unit_keys) for i in range(walks)]
            ends = [s + (span // walks) * unit_keys for s in starts]
            assert starts[0] == origin and ends[-1] == origin + span * unit_keys
            assert all(e == s for e, s in zip(ends, starts[1:]))


def test_chip_ms_per_launch():
    """One context: the launches' own event mean; several in flight: wall time over all launches."""
    import bench
    assert bench.chip_ms_per_launch(1, 280.0, 10, 9.9) == 28.0
    assert bench.chip_ms_per_launch(2, 520.0, 20, 5.0) == 250.0  # 5 s / 20 launches


@pytest.mark.parametrize("seconds,steps,unit_s,quantum,expect", [
    (60, 10, 56.5e-3 / 65536, 65536, 65536 * 107),   # BSGS: 10 steps of ~6 s
    (60, 20, 56.5e-3 / 65536, 65536, 65536 * 54),    # the driver's --steps 20
    (20, 10, 0.57, 1, 4), (20, 10, 0.089, 1, 23),    # rmd160 / xpoint chunks
    (0, 10, 0.57, 1, 1), (60, 10, 0.0, 65536, 65536)])
def test_batch_for_sizes_the_sustained_window(seconds, steps, unit_s, quantum, expect):
    import bench
    b = bench.batch_for(seconds, steps, unit_s, quantum, quantum)
    assert b == expect and b % quantum == 0
    if seconds and unit_s:
        assert b * steps * unit_s >= seconds * 0.999


def test_more_ranks_than_gpus_is_refused_unless_rehearsal():
    import bench
    assert [bench.device_plan(8, r, 8, 8, False) for r in range(8)] == list(range(8))
    with pytest.raises(SystemExit, match="only 1 visible GPU"):
        bench.device_plan(8, 3, 8, 1, False)
    assert bench.device_plan(8, 3, 8, 1, True) == 0
    assert bench.device_plan(4, 3, 4, 2, True) == 1
    with pytest.raises(SystemExit, match="no GPU visible"):
        bench.device_plan(1, 0, 1, 0, True)


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
