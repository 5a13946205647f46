#!/usr/bin/env python3
"""Benchmark of the MI355X keyhunt engine -- one JSON line on rank 0.

Metric (BASELINE.json): "Mkeys/s at 1/2/4/8 GPU (BSGS b125; addr b66); HBM GB/s fraction".
  primary   : -m bsgs -f tests/125.txt -b 125 -k 128  (configs[3]).  A step = one kh_bsgs_scan over
              BASES consecutive bases of 2N keys (N = 2^44) for the puzzle-125 public key, i.e.
              BASES x 32768 giant-step points probed against the 1.84 GB layer-1 bloom, plus the
              host refinement of every first-level candidate.  Keys counted as the reference does
              (2N per base, keyhunt.cpp:4883-4884 / 2871-2874).
  secondary : -m rmd160 -f tests/66.rmd -b 66 -l compress (configs[1]).  A step = one 2^32-key
              N_SEQUENTIAL_MAX chunk; keys counted x2 for -l compress (keyhunt.cpp:2889-2891).
  tertiary  : -m xpoint -f tests/63.pub -b 63 (configs[2]), same chunks, one key per point.
  --config 5: the primary on -m bsgs -f tests/130.txt -b 130 -k 512 (configs[4]) instead.
Ranks split the keyspace (weak scaling, no collective on the data path): rank r walks its own
contiguous run of BSGS base batches and of 2^32-key chunks (r*(W+K) + s), so consecutive calls
continue the same lanes.  The table build (baby steps) is replicated per GPU and not timed; its time is
reported.  torch.distributed (gloo, CPU tensors) provides the barrier and the max over ranks; the
engine owns the GPU through its own HIP stream, synchronised on both sides of the timed region.

roofline: dominant kernel of each leg (the giant-step walk k_walk<7, 2048>; k_walk<11, 2048> and
k_walk<10, 2048> for rmd160 / xpoint), from HIP events the engine records on its own stream around
its launches.  The walks are bound by VALU issue, so "bound" is "valu":
achieved = VALU wave-instructions per launch (rocprofv3 SQ_INSTS_VALU per point, committed under
profiles/, x this run's points per launch) / mean launch time; peak = 1024 SIMDs x 2.4 GHz / 4
cycles: one wave64 VALU instruction per SIMD per quad-cycle, the unit the SQ counters use and the
measured issue cost of the 32-bit multiply-accumulate and carry ops the field math is made of
(4.1-5.5 cycles at 4 waves/SIMD; only add/xor/mov issue in 2).  pmc_valu_issue_frac is the
profiled dispatch's own occupancy of those issue slots, SQ_INSTS_VALU x 4 / (1024 x GRBM_GUI_ACTIVE
/ 8), clock-free (the chip's clock under this load sits below 2.4 GHz: pmc_clock_ghz).  The HBM
side is reported too ("hbm"): algorithmic bytes (BSGS: 64 B per giant point, one random line of the
blocked layer 1; the reference layout's is 128 B) / launch time against 8 TB/s, and
traffic = HBM bytes per launch from the PMC counters with the guide's gfx950 corrections
(tools/pmc_summary.py), or null.
cpu_baseline: rank 0 at N=1 only, on every leg the reference binary built from its own sources
(oracle/_ref/keyhunt, oracle/Makefile.ref; kind "reference") run for --cpu-seconds on the job's CPU
share (cpu_threads), its own last stats line parsed.  BSGS skips the reference's baby-step build:
the engine writes the -S table files in the reference's format (kh_bsgs_save, byte-identical) and the
reference reads them (-S -6).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mkeys/s at 1/2/4/8 GPU (BSGS b125; addr b66); HBM GB/s fraction"
HBM_PEAK_GBS = 8000.0
ALGO_BYTES_PER_GIANT_POINT = {0: 128, 1: 64}      # by layer-1 layout (reference, blocked)
WALK_KERNEL = {0: "k_walk<4, 2048>", 1: "k_walk<7, 2048>"}    # KM_BSGS, KM_BSGSB on 4096-point groups
# 1024 SIMDs x 2.4 GHz / 4 cycles per wave64 VALU instruction (SQ quad-cycle; measured issue cost of
# v_mad_u64_u32 / v_add_co / v_addc_co / v_bitop3 at 4 waves per SIMD: 4.1-5.5 cycles)
SIMDS = 256 * 4
VALU_ISSUE_CYCLES = 4
VALU_PEAK_GIPS = SIMDS * 2.4e9 / VALU_ISSUE_CYCLES / 1e9
RANDOM16_CEILING_GPS = 51.36   # measured random 16-B nontemporal loads/s, 24 GB footprint (profiles/)
PUZZLE125 = "0233709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e"
PUZZLE130 = "03633cbe3ec02b9401c5effa144c5b4d22f87940259634858fc7e59b1c09937852"
# BSGS workloads: --config 4 (the metric's, default) and 5 (BASELINE configs[4], k = 512)
BSGS_CONFIGS = {
    4: {"pub": PUZZLE125, "bits": 125, "k": 128, "bases": 65536,
        "workload": "-m bsgs -f tests/125.txt -b 125 -k 128", "data": "puzzle-125 public key (tests/125.txt)"},
    5: {"pub": PUZZLE130, "bits": 130, "k": 512, "bases": 262144,
        "workload": "-m bsgs -f tests/130.txt -b 130 -k 512", "data": "puzzle-130 public key (tests/130.txt)"},
}
PUZZLE66_RMD = "20d45a6a762535700ce9e0b216e31994335db8a5"
PUZZLE63_X = 0x65ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579  # tests/63.pub
P = 2**256 - 2**32 - 977


def decompress(s: str) -> tuple[int, int]:
    x = int(s[2:], 16)
    y = pow((x * x * x + 7) % P, (P + 1) // 4, P)
    if (y & 1) != (int(s[:2], 16) & 1):
        y = P - y
    return x, y


class Dist:
    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.pg = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.torch, self.dist = torch, dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.world == 1:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def rank_batch(rank: int, warmup: int, steps: int, s: int) -> int:
    """Index of the batch rank `rank` walks at step s (warmup steps included, s < warmup + steps):
    each rank owns one contiguous run of warmup + steps batches, so consecutive steps continue its
    lanes (kh_bsgs_scan / kh_scan keep them across calls that follow on).  Runs of different ranks
    are disjoint and together cover batches 0 .. world*(warmup+steps)-1 (tests/test_dist.py)."""
    return rank * (warmup + steps) + s


def launch_ranks(n: int, argv: list[str], script: str | None = None) -> int:
    """`bench.py --gpus N` started without WORLD_SIZE: start N rank processes of this script (one per
    GPU, RANK/LOCAL_RANK/WORLD_SIZE set, gloo rendezvous on 127.0.0.1), forward rank 0's JSON line and
    return the worst exit status.  Nothing here touches the GPU, so the children start clean."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    out, _ = procs[0].communicate()
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    sys.stdout.write(out)
    sys.stdout.flush()
    return max(abs(rc) for rc in rcs)


def timed(D: Dist, eng, warmup: int, steps: int, step_fn):
    for s in range(warmup):
        step_fn(s)
    eng.synchronize()
    D.barrier()
    eng.kernel_time_reset()
    t0 = time.perf_counter()
    for s in range(steps):
        step_fn(warmup + s)
    eng.synchronize()
    t1 = time.perf_counter()
    D.barrier()
    return D.max(t1 - t0)


def bsgs_leg(D: Dist, eng, args):
    import keyhunt_amd as K
    C = BSGS_CONFIGS[args.config]
    info = eng.bsgs_setup(1 << 44, C["k"], layer1=args.layer1)
    t = time.perf_counter()
    eng.bsgs_build()
    eng.synchronize()
    build_s = time.perf_counter() - t
    q = decompress(C["pub"])
    eng.bsgs_set_targets([q])
    two_n = 2 * info.n
    base0 = 1 << (C["bits"] - 1)
    B = args.bases or C["bases"]

    # rank r walks its own contiguous run of batches, so consecutive steps continue its lanes
    def step(s):
        batch = rank_batch(D.rank, args.warmup, args.steps, s)
        found = eng.bsgs_scan(base0 + batch * B * two_n, B)
        assert not found  # puzzle 125's key lies far from the start of the range

    T = timed(D, eng, args.warmup, args.steps, step)
    la, ms, pts = eng.kernel_time(K.engine.TIME_BSGS)
    keys = D.world * args.steps * B * two_n
    args.bases = B
    pts_launch = pts / la
    ms_launch = ms / la
    bpp = ALGO_BYTES_PER_GIANT_POINT[info.layer1_layout]
    kname = WALK_KERNEL[info.layer1_layout]
    roof = walk_roofline(kname, pts_launch, ms_launch, bpp, la)
    # the probe is one random 16-B load per giant point: its own ceiling is the chip's random-load
    # rate at this footprint (tools/ubench_random2.hip, profiles/r01l_random16B.txt: 24 GB, nt loads)
    rand = {"achieved": pts_launch / (ms_launch / 1e3) / 1e9, "ceiling": RANDOM16_CEILING_GPS, "unit": "G loads/s",
            "frac": pts_launch / (ms_launch / 1e3) / 1e9 / RANDOM16_CEILING_GPS,
            "source": "profiles/r01l_random16B.txt"} if info.layer1_layout == 1 else None
    res = {
        "value": keys / T / 1e6,
        "random_access": rand,
        "ms_per_step": T / args.steps * 1e3,
        "giant_points_per_s": D.world * args.steps * B * info.cycles * 1024 / T,
        "build_seconds": build_s,
        "candidates": eng.bsgs_candidates(),
        "info": info,
        "roofline": roof,
        "q": q,
    }
    return res


def walk_roofline(kname: str, pts_launch: float, ms_launch: float, algo_bytes_per_point: float, launches: int) -> dict:
    """The roofline object of one walk kernel (see the module docstring): VALU issue bound, with the
    HBM side alongside.  Counter-derived figures come from the newest profiles/r*_pmc_summary.json
    holding this kernel and are scaled to this run's points per launch."""
    d = pmc_entry(kname)
    secs = ms_launch / 1e3
    roof = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_GIPS, "unit": "G VALU wave-instr/s", "frac": None,
            "traffic": None, "kernel": kname, "launches": launches, "mean_launch_ms": ms_launch,
            "points_per_launch": pts_launch, "source": d.get("source")}
    if "valu_wave_instructions_per_dispatch" in d:
        wipp = d["valu_wave_instructions_per_dispatch"] / d["points_per_dispatch"]
        a = wipp * pts_launch / secs / 1e9
        roof.update(achieved=a, frac=a / VALU_PEAK_GIPS, valu_wave_instructions_per_point=wipp,
                    valu_lane_instructions_per_point=wipp * 64)
        if d.get("valu_issue_frac"):
            # the profiled dispatch's issue-slot occupancy, in cycles (clock-free; DVFS moves the
            # clock between runs, so frac above is at the nominal 2.4 GHz)
            roof.update(pmc_valu_issue_frac=d["valu_issue_frac"], pmc_clock_ghz=d["effective_clock_ghz"])
    hbm = {"achieved": pts_launch * algo_bytes_per_point / secs / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "algorithmic_bytes_per_point": algo_bytes_per_point}
    hbm["frac"] = hbm["achieved"] / HBM_PEAK_GBS
    if "hbm_bytes_per_point" in d:
        roof["traffic"] = d["hbm_bytes_per_point"] * pts_launch
        hbm.update(traffic_bytes_per_point=d["hbm_bytes_per_point"],
                   traffic_achieved=d["hbm_bytes_per_point"] * pts_launch / secs / 1e9)
        hbm["traffic_frac"] = hbm["traffic_achieved"] / HBM_PEAK_GBS
        for key in ("probe_read_bytes_per_point", "pad_bytes_per_point"):
            if key in d:
                hbm[key] = d[key]
    roof["hbm"] = hbm
    return roof


def pmc_entry(kernel: str) -> dict:
    """This kernel's entry in the newest profiles/r*_pmc_summary.json that has it ({} if none)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_summary.json")), reverse=True):
        d = json.load(open(f)).get(kernel)
        if d:
            return dict(d, source=os.path.relpath(f, REPO))
    return {}


def rmd160_leg(D: Dist, eng, args):
    import keyhunt_amd as K
    eng.set_targets([bytes.fromhex(PUZZLE66_RMD)], bloom_items=1)
    chunk = 1 << 32
    base0 = 1 << 65

    def step(s):
        c = rank_batch(D.rank, args.warmup_rmd, args.steps_rmd, s)
        hits = eng.scan(base0 + c * chunk, chunk, K.KH_MODE_ADDRESS, K.KH_SEARCH_COMPRESS)
        assert not hits

    T = timed(D, eng, args.warmup_rmd, args.steps_rmd, step)
    la, ms, pts = eng.kernel_time(K.engine.TIME_ADDRESS)
    keys = D.world * args.steps_rmd * chunk * 2
    # algorithmic HBM bytes ~0 per key: the 16-B target filter block is L2-resident
    return {"value": keys / T / 1e6, "ms_per_step": T / args.steps_rmd * 1e3,
            "points_per_s_in_kernel": pts / (ms / 1e3),
            "roofline": walk_roofline("k_walk<11, 2048>", pts / la, ms / la, 0, la)}


def xpoint_leg(D: Dist, eng, args):
    """-m xpoint -f tests/63.pub -b 63 (BASELINE configs[2]): X[0..20) probes, one key per point."""
    import keyhunt_amd as K
    eng.set_targets([PUZZLE63_X.to_bytes(32, "big")[:20]], bloom_items=1)
    chunk = 1 << 32
    base0 = 1 << 62

    def step(s):
        c = rank_batch(D.rank, args.warmup_rmd, args.steps_rmd, s)
        hits = eng.scan(base0 + c * chunk, chunk, K.KH_MODE_XPOINT, K.KH_SEARCH_COMPRESS)
        assert not hits

    T = timed(D, eng, args.warmup_rmd, args.steps_rmd, step)
    la, ms, pts = eng.kernel_time(K.engine.TIME_XPOINT)
    keys = D.world * args.steps_rmd * chunk
    return {"value": keys / T / 1e6, "ms_per_step": T / args.steps_rmd * 1e3,
            "points_per_s_in_kernel": pts / (ms / 1e3),
            "roofline": walk_roofline("k_walk<10, 2048>", pts / la, ms / la, 0, la)}


def cpu_host() -> dict:
    """The host the CPU baseline ran on: model and CPU count (lscpu), the CPUs this process may use,
    and the threads the baseline used.  On the pool's GPU boxes a one-GPU job's CPU share is 16
    threads (OMP_NUM_THREADS, set by the box) of a much larger machine, so the baseline uses that
    share; `per_thread` values let the reader scale it to any core count."""
    info = {"machine_cpus": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for key, name in (("Model name", "model"), ("Socket(s)", "sockets"), ("Core(s) per socket", "cores_per_socket"),
                          ("Thread(s) per core", "threads_per_core")):
            m = re.search(rf"^{re.escape(key)}:\s*(.+)$", out, re.M)
            if m:
                info[name] = m.group(1).strip()
    except Exception:
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity_cpus"] = os.cpu_count()
    info["threads_used"] = cpu_threads()
    return info


def cpu_threads() -> int:
    """The job's CPU share: OMP_NUM_THREADS when the environment sets it (16 per GPU on the pool's
    boxes), else every CPU this process may run on."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(aff, int(share))) if share.isdigit() and int(share) > 0 else max(1, aff)


REF_BIN = os.path.join(REPO, "oracle", "_ref", "keyhunt")


def run_reference(argv: list[str], files: list[str], seconds: float, setup=None):
    """Run the reference CLI (oracle/_ref/keyhunt, built from /root/reference's sources by
    oracle/Makefile.ref) in a scratch directory under /tmp for `seconds` after its tables are ready,
    with every thread of the job's CPU share, and parse its own last stats line
    ("Total N keys in S seconds", keyhunt.cpp:2906-2946).  `setup(dir)` may write table files first."""
    if not os.path.exists(REF_BIN):
        return None
    thr = cpu_threads()
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for f in files:
            shutil.copy(os.path.join(REPO, "tests", "golden", "data", f), td)
        if setup:
            setup(td)
        cmd = [REF_BIN] + argv + ["-t", str(thr), "-s", "5", "-q"]
        p = subprocess.Popen(cmd, cwd=td, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
        out = b""
        t0 = time.time()
        os.set_blocking(p.stdout.fileno(), False)
        last = None
        while time.time() - t0 < seconds + 120:
            time.sleep(0.5)
            try:
                chunk = p.stdout.read()
            except Exception:
                chunk = None
            if chunk:
                out += chunk
            rates = re.findall(rb"Total (\d+) keys in (\d+) seconds", out)
            if rates:
                last = tuple(map(int, rates[-1]))
                if last[1] >= seconds:
                    break
            if p.poll() is not None:
                break
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if not last or last[1] == 0:
        return None
    keys, secs = last
    return {"value": keys / secs / 1e6, "unit": "Mkeys/s", "cores": thr, "kind": "reference",
            "per_thread": keys / secs / 1e6 / thr, "host": cpu_host(),
            "sample": f"oracle/_ref/keyhunt {' '.join(argv)} -t {thr}: {keys} keys in {secs} s (the reference's "
                      f"own stats line, keys counted as it counts them)"}


def cpu_baseline_bsgs(eng, C: dict, seconds: float):
    """The reference's BSGS giant-step loop (thread_process_bsgs, keyhunt.cpp:4549-4888) on the host,
    on the same workload (-b bits -k K from 2^(bits-1)).  Its 120-s-per-core baby-step build is
    skipped: the engine writes the four -S table files (kh_bsgs_save: the reference's format, byte
    for byte, tests/test_gpu_tables.py) and the reference reads them (-S -6, keyhunt.cpp:1983-2240)."""
    pub = {125: "125.txt", 130: "130.txt"}[C["bits"]]
    return run_reference(["-m", "bsgs", "-f", pub, "-b", str(C["bits"]), "-k", str(C["k"]), "-S", "-6"], [pub],
                         seconds, setup=lambda d: eng.bsgs_save(d))


def cpu_baseline_rmd160(seconds: float):
    return run_reference(["-m", "rmd160", "-f", "66.rmd", "-b", "66", "-l", "compress"], ["66.rmd"], seconds)


def cpu_baseline_xpoint(seconds: float):
    return run_reference(["-m", "xpoint", "-f", "63.pub", "-b", "63"], ["63.pub"], seconds)


def main():
    if "WORLD_SIZE" not in os.environ:
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        n = pre.parse_known_args()[0].gpus
        if n > 1:
            sys.exit(launch_ranks(n, sys.argv[1:]))
    # stdout carries exactly one JSON line (rank 0); native libraries (gloo, HIP) may print on fd 1,
    # so fd 1 is pointed at stderr for the run and the JSON goes to the saved descriptor.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, choices=sorted(BSGS_CONFIGS),
                    help="BSGS workload: 4 = b125 k128 (the metric's), 5 = b130 k512")
    ap.add_argument("--bases", type=int, default=0, help="BSGS bases (of 2N keys) per step per GPU (0: per config)")
    ap.add_argument("--steps-rmd", type=int, default=None)
    ap.add_argument("--warmup-rmd", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--layer1", type=int, default=1, help="BSGS layer-1 layout: 1 blocked (default), 0 reference")
    args = ap.parse_args()
    args.steps_rmd = args.steps if args.steps_rmd is None else args.steps_rmd
    args.warmup_rmd = args.warmup if args.warmup_rmd is None else args.warmup_rmd

    import keyhunt_amd as K
    D = Dist()
    if args.gpus != D.world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={D.world}: launch one rank per GPU")
    ndev = K.device_count()
    # one process per GPU; on a box with fewer GPUs than ranks (rehearsal) ranks share devices
    eng = K.Engine(D.local % max(1, ndev))
    prim = bsgs_leg(D, eng, args)
    sec = None if args.no_secondary else rmd160_leg(D, eng, args)
    ter = None if args.no_secondary else xpoint_leg(D, eng, args)
    cpu_b = cpu_r = cpu_x = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline:
        cpu_b = cpu_baseline_bsgs(eng, BSGS_CONFIGS[args.config], args.cpu_seconds)
        if not args.no_secondary:
            cpu_r = cpu_baseline_rmd160(args.cpu_seconds)
            cpu_x = cpu_baseline_xpoint(args.cpu_seconds)
    eng.close()
    D.barrier()
    if D.rank == 0:
        info = prim["info"]
        line = {
            "metric": METRIC, "value": prim["value"], "unit": "Mkeys/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": prim["ms_per_step"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32",
            "data": f"synthetic: {BSGS_CONFIGS[args.config]['data']}, sequential bases from 2^{BSGS_CONFIGS[args.config]['bits'] - 1}",
            "config": {"workload": BSGS_CONFIGS[args.config]["workload"], "n": info.n, "k": BSGS_CONFIGS[args.config]["k"], "m": info.m,
                       "layer1_layout": "blocked" if info.layer1_layout == 1 else "reference",
                       "bases_per_step": args.bases, "giant_points_per_step": args.bases * info.cycles * 1024,
                       "parallelism": f"keyspace split x{D.world} (no collective)"},
            "giant_points_per_s": prim["giant_points_per_s"],
            "build_seconds": prim["build_seconds"],
            "first_level_candidates": prim["candidates"],
            "roofline": prim["roofline"],
            "random_access": prim["random_access"],
            "cpu_baseline": cpu_b,
        }
        if sec:
            line["secondary"] = {"workload": "-m rmd160 -f tests/66.rmd -b 66 -l compress", "value": sec["value"],
                                 "unit": "Mkeys/s", "ms_per_step": sec["ms_per_step"], "steps": args.steps_rmd,
                                 "points_per_s_in_kernel": sec["points_per_s_in_kernel"],
                                 "roofline": sec["roofline"], "cpu_baseline": cpu_r}
        if ter:
            line["tertiary"] = {"workload": "-m xpoint -f tests/63.pub -b 63", "value": ter["value"],
                                "unit": "Mkeys/s", "ms_per_step": ter["ms_per_step"], "steps": args.steps_rmd,
                                "points_per_s_in_kernel": ter["points_per_s_in_kernel"],
                                "roofline": ter["roofline"], "cpu_baseline": cpu_x}
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    D.close()


if __name__ == "__main__":
    main()
