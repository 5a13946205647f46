#!/usr/bin/env python3
"""Benchmark of the MI355X keyhunt engine -- one JSON line on rank 0.

Metric (BASELINE.json): "Mkeys/s at 1/2/4/8 GPU (BSGS b125; addr b66); HBM GB/s fraction".
  primary   : -m bsgs -f tests/125.txt -b 125 -k 128  (configs[3]).  A step = one kh_bsgs_scan over
              B consecutive bases of 2N keys (N = 2^44) for the puzzle-125 public key, i.e.
              B x 32768 giant-step points probed against the layer-1 filter, plus the second check of
              every first-level candidate.  Keys counted as the reference does (2N per base,
              keyhunt.cpp:4883-4884 / 2871-2874).
  secondary : -m rmd160 -f tests/66.rmd -b 66 -l compress (configs[1]).  A step = C consecutive
              2^32-key N_SEQUENTIAL_MAX chunks (one kh_scan each); keys counted x2 for -l compress
              (keyhunt.cpp:2889-2891).
  tertiary  : -m xpoint -f tests/63.pub -b 63 (configs[2]), same chunks, one key per point.
  --config 5: the primary on -m bsgs -f tests/130.txt -b 130 -k 512 (configs[4]) instead.

Sustained measurement (throughput runs of >= 60 s after warm-up): the batch of a step
(B bases, C chunks) is sized from the last warm-up step so that the K timed steps last --seconds
(primary, default 60) and --seconds-secondary (default 20) per address-family leg; the line reports
the rate of the first and the last quarter of the timed steps, each with its kernel time per launch,
the board's gfx clock and socket power (amdsmi), and over the whole timed region the board's own
counters (BoardSampler): mean socket power from the energy accumulator, the power cap, the share of
the time spent at the package power limit (ppt_residency_frac, "power_capped") and points per joule.

Parity at full size: after each leg's timed loop (outside it), the same engine with the same tables
scans the SURVEY.md 8c known-answer window of that workload and must find the reference's key
("known_answer" per leg); bench.py exits 3 on a mismatch, after printing the line.

Ranks split the keyspace (weak scaling, no collective on the data path): rank r walks its own
contiguous region starting at r * span units (rank_origin), so consecutive steps continue the same
lanes.  One process per GPU: more ranks than visible devices is refused unless --rehearse (ranks then
share devices and the line says so); the line reports the distinct devices (PCI bus ids) the ranks
used and every rank's own rate.  The table build is replicated per GPU and not timed; its time is
reported.  torch.distributed (gloo, CPU tensors) provides the barrier and the max over ranks; the
engine owns the GPU through its own HIP stream, synchronised on both sides of the timed region.

Walks in flight (--walks, --walks-secondary; Walks): each leg may drive S contexts on its GPU, each
with its own stream and host thread, walking its own contiguous part of the rank region
(walk_origin).  Default S = 1 for every leg: the configuration the CLI and the INTEGRATION.md binding
run.  With S > 1 the launches overlap, so the roofline prices the chip's time per launch (timed wall /
all launches, chip_ms_per_launch) and reports the launches' own event mean beside it
(event_mean_launch_ms, which a rocprofv3 kernel trace of the run agrees with).

roofline: dominant kernel of each leg (the giant-step walk k_walk<7, 2048>; k_walk<11, 2048> and
k_walk<10, 2048> for rmd160 / xpoint), from HIP events the engine records on its own stream around
its launches.  The walks are bound by VALU issue, so "bound" is "valu":
achieved = VALU wave-instructions per launch (rocprofv3 SQ_INSTS_VALU per point, committed under
profiles/, x this run's points per launch) / mean launch time.  Two ceilings, both upper bounds:
  peak / frac   1024 SIMDs x 2.4 GHz / 2 cycles: the hardware's wave64 VALU issue on a SIMD-32
                (MI355X_MICROARCH.md), which only full-rate instructions reach;
  frac_mix      the kernel's own instruction mix per point at the issue floor of each instruction
                (2 / 4 cycles per full- / half-rate wave64 instruction, s_nop at its measured in-situ
                cost, dual-issued instructions free; tools/valu_mix.py -> profiles/r*_valu_mix.json)
                at the clock the board reported over the leg's timed region.
The HBM side is reported too ("hbm"): algorithmic bytes (BSGS: 64 B per giant point, one random line
of the blocked layer 1; the reference layout's is 128 B) / launch time against 8 TB/s,
and traffic = HBM bytes per launch from the PMC counters with the guide's gfx950 corrections
(tools/pmc_summary.py), or null.
cpu_baseline: rank 0 at N=1 only, on every leg the reference binary built from its own sources with
its own optimisation flags (oracle/_ref/keyhunt_fast, oracle/Makefile.ref; kind "reference"), run for
--cpu-seconds-primary (BSGS) / --cpu-seconds (rmd160, xpoint), 60 s each, of its own stats clock on the
job's CPU share (cpu_threads: "value", "threads"), then for --cpu-seconds-per-core (30 s) with -t 1
("per_core"), its own last stats line parsed each time; the host's sockets, physical cores and threads
per core come from lscpu.  BSGS skips the reference's
baby-step build: the engine writes the -S table files in the reference's format (kh_bsgs_save,
byte-identical) and the reference reads them (-S -6).

The line ends with "legs": one compact object per leg (value, unit, known-answer match, roofline frac,
the CPU baseline's value and sample seconds), so the three legs' numbers sit in the last bytes of the
line, which a runner that keeps only the tail of stdout still holds.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mkeys/s at 1/2/4/8 GPU (BSGS b125; addr b66); HBM GB/s fraction"
HBM_PEAK_GBS = 8000.0
ALGO_BYTES_PER_GIANT_POINT = {0: 128, 1: 64}      # by layer-1 layout (reference, blocked)
WALK_KERNEL = {0: "k_walk<4, 2048>", 1: "k_walk<7, 2048>"}    # KM_BSGS, KM_BSGSB on 4096-point groups
SIMDS = 256 * 4
NOMINAL_GHZ = 2.4
# the hardware's VALU issue peak: 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction on a SIMD-32
# (MI355X_MICROARCH.md); only full-rate instructions reach it, the walks' multiply-adds and carry ops
# take 4 cycles (profiles/r04_valu_mix.json prices the mix: frac_mix)
VALU_PEAK_GIPS = SIMDS * NOMINAL_GHZ / 2
RANDOM16_CEILING_GPS = 51.36   # measured random 16-B nontemporal loads/s, 24 GB footprint (profiles/)
PUZZLE125 = "0233709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e"
PUZZLE130 = "03633cbe3ec02b9401c5effa144c5b4d22f87940259634858fc7e59b1c09937852"
# BSGS workloads: --config 4 (the metric's, default) and 5 (BASELINE configs[4], k = 512), each with
# the SURVEY.md 8c known-answer window (verified with the reference CLI) checked after the timed loop
BSGS_CONFIGS = {
    4: {"pub": PUZZLE125, "bits": 125, "k": 128, "bases": 65536,
        "workload": "-m bsgs -f tests/125.txt -b 125 -k 128", "data": "puzzle-125 public key (tests/125.txt)",
        "ka": (0x1c533b6bb7f0804e0995fe0000000000, 0x1c533b6bb7f0804e09963e0000000000,
               0x1c533b6bb7f0804e09960225e44877ac)},
    5: {"pub": PUZZLE130, "bits": 130, "k": 512, "bases": 262144,
        "workload": "-m bsgs -f tests/130.txt -b 130 -k 512", "data": "puzzle-130 public key (tests/130.txt)",
        "ka": (0x33e7665705359f04f28b8880000000000, 0x33e7665705359f04f28b8c80000000000,
               0x33e7665705359f04f28b88cf897c603c9)},
}
PUZZLE66_RMD = "20d45a6a762535700ce9e0b216e31994335db8a5"
PUZZLE63_X = 0x65ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579  # tests/63.pub
# known-answer windows of the address-family legs (reference CLI): (start, keys, key)
KA_RMD160 = (0x2832ed74f2b000000, 1 << 24, 0x2832ed74f2b5e35ee)
KA_XPOINT = (0x7cce5efdac000000, 1 << 24, 0x7cce5efdaccf6808)
# per-rank regions (rank_origin): BSGS bases, address-family 2^32-key chunks
RANK_SPAN_BASES = 1 << 40
RANK_SPAN_CHUNKS = 1 << 24
CHUNK = 1 << 32
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
        self.local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
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

    def gather(self, obj) -> list:
        """Every rank's obj, in rank order (on every rank)."""
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def rank_origin(rank: int, span: int) -> int:
    """First unit (BSGS base / 2^32-key chunk, counted from the workload's start) of rank `rank`'s
    region: each rank walks one contiguous run from there, warm-up and timed steps alike, so
    consecutive calls continue its lanes (kh_bsgs_scan / kh_scan keep them across calls that follow
    on).  Regions of different ranks are disjoint as long as a rank walks fewer than `span` units,
    which the legs check (tests/test_dist.py)."""
    return rank * span


def walk_origin(origin: int, walk: int, walks: int, span: int, unit_keys: int) -> int:
    """First key of walk `walk`'s part of a rank region that starts at key `origin` and holds `span`
    units of `unit_keys` keys: the region is cut into `walks` contiguous parts, one per context, so each
    context's consecutive calls continue its own lanes and no two contexts cover the same key."""
    return origin + walk * (span // walks) * unit_keys


class Walks:
    """`walks` contexts on one device (kh_open each: own HIP stream, own tables, inversion pads and
    lane states), each driven by its own host thread, so up to `walks` walk launches are in flight on
    the chip at once.  One launch's tail and the phases in which all its waves wait on the same thing
    (pad stores, the batch inversion, the probes) leave issue slots idle that the other context's
    waves fill (profiles/r03t_rehearse2_one_gpu.json).  ctypes drops the GIL
    for the duration of every kh_* call, so the threads' calls overlap."""

    def __init__(self, K, device: int, walks: int):
        from concurrent.futures import ThreadPoolExecutor
        self.engs = [K.Engine(device) for _ in range(walks)]
        self.pool = ThreadPoolExecutor(walks) if walks > 1 else None

    def __len__(self):
        return len(self.engs)

    def head(self, n: int) -> "Walks":
        """The first n contexts as a set of their own (same threads), for a leg that walks fewer."""
        v = Walks.__new__(Walks)
        v.engs, v.pool = self.engs[:n], self.pool if n > 1 else None
        return v

    def each(self, fn) -> list:
        """fn(i, engine) on every context, concurrently; results in context order."""
        if self.pool is None:
            return [fn(0, self.engs[0])]
        return [f.result() for f in [self.pool.submit(fn, i, e) for i, e in enumerate(self.engs)]]

    def synchronize(self) -> None:
        for e in self.engs:
            e.synchronize()

    def kernel_time_reset(self) -> None:
        for e in self.engs:
            e.kernel_time_reset()

    def kernel_time(self, kind: int) -> tuple[int, float, int]:
        """Launches, event ms and points summed over the contexts."""
        t = [e.kernel_time(kind) for e in self.engs]
        return sum(x[0] for x in t), sum(x[1] for x in t), sum(x[2] for x in t)

    def close(self) -> None:
        for e in self.engs:
            e.close()
        if self.pool:
            self.pool.shutdown()


# walk contexts per GPU, per leg (bench.py --walks / --walks-secondary): one, as the CLI and the
# INTEGRATION.md binding open.  Round 3 ran the address legs on two contexts, whose launches filled each
# other's phases (xpoint +17 %); since round 4 one context's launch holds 2^20 lanes, four waves per
# wave slot, which gets the same (kh_kernels.h KH_LANES_HB, profiles/r04a_geom_ab.json)
WALKS_BSGS = 1
WALKS_ADDRESS = 1


def batch_for(seconds: float, steps: int, unit_s: float, quantum: int, floor: int) -> int:
    """Units per step so that `steps` steps of unit_s seconds per unit last about `seconds`: a
    multiple of `quantum`, at least `floor`."""
    if seconds <= 0 or unit_s <= 0 or steps <= 0:
        return floor
    want = seconds / steps / unit_s
    return max(floor, int(-(-want // quantum)) * quantum)


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


def device_plan(world: int, local_rank: int, local_world: int, ndev: int, rehearse: bool) -> int:
    """The device this rank uses: its local rank.  One process per GPU, so more local ranks than
    visible devices is refused unless `rehearse` (ranks then share devices round-robin and the line
    reports it: devices_used, rehearsal)."""
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    if local_world > ndev and not rehearse:
        raise SystemExit(f"bench.py: {local_world} ranks on this node but only {ndev} visible GPU(s): one rank per "
                         f"GPU (pass --rehearse to stack ranks on fewer devices; the line then says so)")
    return local_rank % ndev


def pci_bus_id(device: int) -> str | None:
    """PCI bus id of HIP device `device`, from the HIP runtime the engine itself loaded."""
    try:
        path = None
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    path = line.split()[-1]
                    break
        hip = ctypes.CDLL(path or "libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return None
        return buf.value.decode().lower()
    except Exception:
        return None


def _num(v) -> float | None:
    return float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) and v != 0xFFFF else None


class BoardSampler:
    """The board's own view of a run (amdsmi, device with bus id `bdf`; the only device when there is
    one): gfx clock (MHz, mean over the XCDs' current_gfxclks) and socket power (W) sampled every
    `period` s in a thread, plus counter snapshots (`snapshot`) whose differences (`between`) give

      * mean socket power from the energy accumulator (amdsmi_get_energy_count, its own resolution);
      * the share of the interval spent at the package power limit (PPT), at a thermal limit
        (socket / HBM / VR) and under PROCHOT, from the firmware's residency accumulators over its
        accumulation counter (gpu_metrics ppt_residency_acc etc.): 1.0 = limited the whole time;
      * the power cap in force (amdsmi_get_power_cap_info, W).

    Board clocks run a few % above the in-kernel clock (MI355X_MICROARCH.md, DVFS give-back): a
    trend indicator beside the kernel times, not a cycle count."""

    RESIDENCY = ("ppt_residency_acc", "socket_thm_residency_acc", "hbm_thm_residency_acc", "vr_thm_residency_acc",
                 "prochot_residency_acc")
    # other gpu_metrics fields averaged over a window when the board reports them (MHz / %)
    EXTRA = ("current_uclk", "current_fclk", "current_socclks", "average_umc_activity", "average_gfx_activity")

    def __init__(self, bdf: str | None, period: float = 0.25):
        self.samples: list[tuple[float, float]] = []        # (t, gfx MHz)
        self.power_samples: list[tuple[float, float]] = []  # (t, socket W)
        self.extra_samples: dict[str, list[tuple[float, float]]] = {}
        self.error = None
        self._stop = threading.Event()
        self._h = None
        self._period = period
        self._lock = threading.Lock()
        try:
            import amdsmi
            self._amdsmi = amdsmi
            amdsmi.amdsmi_init()
            hs = amdsmi.amdsmi_get_processor_handles()
            for h in hs:
                b = str(amdsmi.amdsmi_get_gpu_device_bdf(h)).lower()
                if bdf and (b == bdf or b.endswith(bdf.split(":", 1)[-1]) or bdf.endswith(b.split(":", 1)[-1])):
                    self._h = h
                    break
            if self._h is None and len(hs) == 1:
                self._h = hs[0]
            if self._h is None:
                self.error = f"no amdsmi device with bus id {bdf}"
        except Exception as e:  # amdsmi absent or not permitted: the line says why
            self.error = f"amdsmi: {e!r}"[:200]
        self._t = None

    def _metrics(self) -> dict:
        with self._lock:
            return self._amdsmi.amdsmi_get_gpu_metrics_info(self._h)

    @staticmethod
    def _clock_of(m: dict) -> float | None:
        v = m.get("current_gfxclks")
        if isinstance(v, list):
            vals = [x for x in v if isinstance(x, (int, float)) and 0 < x < 10000]
            if vals:
                return sum(vals) / len(vals)
        for key in ("current_gfxclk", "average_gfxclk_frequency"):
            x = _num(m.get(key))
            if x and 0 < x < 10000:
                return x
        return None

    def _energy(self) -> tuple[float, float] | None:
        """(joules, resolution in J) from the energy accumulator."""
        try:
            with self._lock:
                e = self._amdsmi.amdsmi_get_energy_count(self._h)
            res = float(e["counter_resolution"]) * 1e-6  # µJ per count
            return float(e["energy_accumulator"]) * res, res
        except Exception:
            return None

    def _run(self):
        while not self._stop.is_set():
            try:
                m = self._metrics()
                t = time.perf_counter()
                c = self._clock_of(m)
                if c:
                    self.samples.append((t, c))
                p = _num(m.get("current_socket_power"))
                if p:
                    self.power_samples.append((t, p))
                # memory / fabric clocks and memory-controller activity, where gpu_metrics has them
                for k in self.EXTRA:
                    v = m.get(k)
                    if isinstance(v, list):
                        v = [x for x in v if isinstance(x, (int, float)) and 0 < x < 65535]
                        v = sum(v) / len(v) if v else None
                    else:
                        v = _num(v)
                    if v is not None and 0 <= v < 65535:
                        self.extra_samples.setdefault(k, []).append((t, v))
            except Exception as e:
                self.error = f"amdsmi read: {e!r}"[:200]
                return
            self._stop.wait(self._period)

    def start(self):
        if self._h is not None:
            self._t = threading.Thread(target=self._run, daemon=True)
            self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t:
            self._t.join(timeout=5)

    def mean(self, t0: float, t1: float) -> float | None:
        v = [c for t, c in self.samples if t0 <= t <= t1]
        return sum(v) / len(v) if v else None

    def mean_power(self, t0: float, t1: float) -> float | None:
        v = [c for t, c in self.power_samples if t0 <= t <= t1]
        return sum(v) / len(v) if v else None

    def snapshot(self) -> dict | None:
        """Counter values now (perf_counter time, energy, residency accumulators)."""
        if self._h is None:
            return None
        try:
            m = self._metrics()
        except Exception as e:
            self.error = f"amdsmi read: {e!r}"[:200]
            return None
        s = {"t": time.perf_counter(), "acc": _num(m.get("accumulation_counter"))}
        for k in self.RESIDENCY:
            s[k] = _num(m.get(k))
        en = self._energy()
        s["energy_j"], s["energy_res_j"] = en if en else (None, None)
        return s

    def between(self, a: dict | None, b: dict | None) -> dict | None:
        """Mean power, power-limit residency and board clock between two snapshots."""
        if not a or not b:
            return None
        dt = b["t"] - a["t"]
        out = {"seconds": dt, "board_gfxclk_mhz": self.mean(a["t"], b["t"]),
               "socket_power_w_sampled": self.mean_power(a["t"], b["t"])}
        for k, v in self.extra_samples.items():
            w = [c for t, c in v if a["t"] <= t <= b["t"]]
            if w:
                out[k] = sum(w) / len(w)
        if a.get("energy_j") is not None and b.get("energy_j") is not None and dt > 0:
            out["socket_power_w"] = (b["energy_j"] - a["energy_j"]) / dt
        if a.get("acc") is not None and b.get("acc") is not None and b["acc"] > a["acc"]:
            da = b["acc"] - a["acc"]
            out["accumulation_counts"] = da
            for k in self.RESIDENCY:
                if a.get(k) is not None and b.get(k) is not None:
                    out[k.replace("_acc", "_frac")] = (b[k] - a[k]) / da
        cap = self.power_cap_w()
        if cap:
            out["power_cap_w"] = cap
            if out.get("socket_power_w"):
                out["power_over_cap"] = out["socket_power_w"] / cap
        return out

    def power_cap_w(self) -> float | None:
        try:
            with self._lock:
                c = self._amdsmi.amdsmi_get_power_cap_info(self._h)
            v = _num(c.get("power_cap"))
            return v / 1e6 if v and v > 1e5 else v  # reported in µW
        except Exception:
            return None

    def info(self) -> dict:
        out = {"error": self.error, "samples": len(self.samples), "power_samples": len(self.power_samples)}
        if self._h is not None:
            try:
                with self._lock:
                    out["power_cap_info"] = self._amdsmi.amdsmi_get_power_cap_info(self._h)
                    out["power_info"] = self._amdsmi.amdsmi_get_power_info(self._h)
            except Exception as e:
                out["power_cap_error"] = repr(e)[:200]
        return out


ClockSampler = BoardSampler


def timed(D: Dist, eng, steps: int, step_fn, units_per_step: int, kind: int, clock: BoardSampler | None):
    """K timed steps bracketed by barrier + synchronize; returns (max-over-ranks seconds, t0, t1,
    per-step records (wall end, cumulative kernel ms and launches) for the quarter analysis, the
    board's counters between t0 and t1 (BoardSampler.between: power, power-limit residency, clock))."""
    eng.synchronize()
    D.barrier()
    eng.kernel_time_reset()
    recs = []
    b0 = clock.snapshot() if clock else None
    t0 = time.perf_counter()
    for s in range(steps):
        step_fn(s)
        la, ms, _ = eng.kernel_time(kind)
        recs.append((time.perf_counter(), ms, la))
    eng.synchronize()
    t1 = time.perf_counter()
    b1 = clock.snapshot() if clock else None
    D.barrier()
    return D.max(t1 - t0), t0, t1, recs, (clock.between(b0, b1) if clock else None)


def quarters(t0: float, recs: list, units_per_step: int, keys_per_unit: float, clock: BoardSampler | None,
             board: dict | None = None, points_per_s: float | None = None) -> dict | None:
    """Rate of the first and the last quarter of the timed steps (keys/s from their wall time), their
    kernel ms per launch, the mean board clock and socket power while they ran; and over the whole
    timed region (`board`, BoardSampler.between) the mean power, the share of it spent at the package
    power limit (ppt_residency_frac) and the points per joule."""
    K = len(recs)
    if K < 4:
        return None
    q = K // 4
    out = {}
    for name, a, b in (("first_quarter", 0, q), ("last_quarter", K - q, K)):
        ts = t0 if a == 0 else recs[a - 1][0]
        ms0, la0 = (0.0, 0) if a == 0 else (recs[a - 1][1], recs[a - 1][2])
        te, ms1, la1 = recs[b - 1]
        out[name] = {"steps": [a, b], "mkeys_per_s": (b - a) * units_per_step * keys_per_unit / (te - ts) / 1e6,
                     "kernel_ms_per_launch": (ms1 - ms0) / max(1, la1 - la0),
                     "board_gfxclk_mhz": clock.mean(ts, te) if clock else None,
                     "socket_power_w": clock.mean_power(ts, te) if clock else None}
    f, l = out["first_quarter"], out["last_quarter"]
    out["last_over_first"] = l["mkeys_per_s"] / f["mkeys_per_s"]
    if board:
        out["board"] = board
        if points_per_s and board.get("socket_power_w"):
            out["points_per_joule"] = points_per_s / board["socket_power_w"]
        ppt = board.get("ppt_residency_frac")
        if ppt is not None:
            out["power_capped"] = {"ppt_residency_frac": ppt, "socket_power_w": board.get("socket_power_w"),
                                   "power_cap_w": board.get("power_cap_w"),
                                   "verdict": "power-capped" if ppt >= 0.5 else "partly power-capped" if ppt >= 0.1
                                   else "not power-capped"}
    return out


def progress(msg: str) -> None:
    """One line on stderr (rank 0) so a long leg shows it is alive."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def bsgs_leg(D: Dist, W: Walks, args, clock):
    import keyhunt_amd as K
    C = BSGS_CONFIGS[args.config]
    S = len(W)
    info = W.each(lambda i, e: e.bsgs_setup(1 << 44, C["k"], layer1=args.layer1))[0]
    t = time.perf_counter()
    W.each(lambda i, e: (e.bsgs_build(), e.synchronize()))
    build_s = time.perf_counter() - t
    progress(f"BSGS tables built in {build_s:.2f} s (k = {C['k']}, {S} context(s))")
    q = decompress(C["pub"])
    W.each(lambda i, e: e.bsgs_set_targets([q]))
    two_n = 2 * info.n
    origin = (1 << (C["bits"] - 1)) + rank_origin(D.rank, RANK_SPAN_BASES) * two_n
    B0 = args.bases or C["bases"]
    assert B0 % S == 0, "--bases must be a multiple of --walks"
    walked = 0

    def run(nb):
        # nb bases per step in all, nb / S per context, each in its own part of the rank's region
        nonlocal walked
        per = nb // S
        assert walked + per <= RANK_SPAN_BASES // S, "rank region exhausted"
        found = W.each(lambda i, e: e.bsgs_scan(walk_origin(origin, i, S, RANK_SPAN_BASES, two_n) + walked * two_n, per))
        walked += per
        assert not any(found)  # puzzle 125's (130's) key lies far from the start of the range

    # warm-up steps large enough for the engine's placement calibration (a context's first call of
    # >= 2^23 walk groups times two inversion-pad placements against each other in four parts, DESIGN.md
    # §2 "Placement"), so it happens here and not in the timed region; 2^24 groups: parts of 2^34 points
    gpb = max(1, info.cycles * 1024 // 4096)
    Bw = max(B0, -(-(8 << 21) // gpb) * S) if args.warmup else B0
    last = 0.0
    for s in range(args.warmup):
        t = time.perf_counter()
        run(Bw)
        last = time.perf_counter() - t
    B = int(D.max(batch_for(args.seconds, args.steps, last / Bw, B0, B0) if args.warmup else B0))
    # whole tiles of the engine's 2^21 lanes (2^18 bases of 8 groups at k = 128): consecutive steps
    # then continue their lanes, and no ragged last round walks unprobed points
    lanes = int(os.environ.get("KH_BSGS_LANES", 1 << 21))
    tile = lanes // max(1, info.cycles * 1024 // 4096) * S
    if not args.bases and B >= tile:
        B = max(tile, (B + tile // 2) // tile * tile)
    progress(f"BSGS warm-up done; timing {args.steps} steps of {B} bases")
    T, t0, t1, recs, board = timed(D, W, args.steps, lambda s: run(B), B, K.engine.TIME_BSGS, clock)
    progress(f"BSGS timed region {T:.1f} s; known-answer window next")
    lanes_pick, rate_hi, rate_lo = W.engs[0].bsgs_geometry()
    cal_done, cal_rates = W.engs[0].bsgs_placement()
    la, ms, pts = W.kernel_time(K.engine.TIME_BSGS)
    my_pts_s = args.steps * B * info.cycles * 1024 / (recs[-1][0] - t0)
    # known answer (outside the timed region, same engine and tables): SURVEY.md 8c
    ka_lo, ka_hi, ka_key = C["ka"]
    ka_found = W.engs[0].bsgs_scan(ka_lo, (ka_hi - ka_lo) // two_n)
    keys = D.world * args.steps * B * two_n
    pts_launch = pts / la
    ms_launch = chip_ms_per_launch(S, ms, la, t1 - t0)
    bpp = ALGO_BYTES_PER_GIANT_POINT[info.layer1_layout]
    kname = WALK_KERNEL[info.layer1_layout]
    roof = walk_roofline(kname, pts_launch, ms_launch, bpp, la, walks=S, event_ms=ms / la,
                         clock_mhz=(board or {}).get("board_gfxclk_mhz"))
    # the probe is one random 16-B load per giant point: its own ceiling is the chip's random-load
    # rate at this footprint (tools/ubench_random2.hip, profiles/r01l_random16B.txt: 24 GB, nt loads)
    rand = {"achieved": pts_launch / (ms_launch / 1e3) / 1e9, "ceiling": RANDOM16_CEILING_GPS, "unit": "G loads/s",
            "frac": pts_launch / (ms_launch / 1e3) / 1e9 / RANDOM16_CEILING_GPS,
            "source": "profiles/r01l_random16B.txt"} if info.layer1_layout == 1 else None
    return {
        "value": keys / T / 1e6,
        "random_access": rand,
        "ms_per_step": T / args.steps * 1e3,
        "seconds_timed": T,
        "bases_per_step": B,
        "placement_calibration": {"complete": cal_done, "lanes": lanes_pick,
                                  "pad_giant_points_per_s_kept": cal_rates[0], "pad_other": cal_rates[1],
                                  "layer1_giant_points_per_s_kept": cal_rates[2], "layer1_other": cal_rates[3]},
        "giant_points_per_s": D.world * args.steps * B * info.cycles * 1024 / T,
        "rank_giant_points_per_s": my_pts_s,
        "build_seconds": build_s,
        "candidates": sum(e.bsgs_candidates() for e in W.engs),
        "info": info,
        "roofline": roof,
        "sustained": quarters(t0, recs, B, two_n, clock, board, my_pts_s),
        "known_answer": {"window": f"{ka_lo:x}:{ka_hi:x}", "expected": f"{ka_key:x}",
                         "found": [f"{k:x}" for _, k in ka_found], "match": [k for _, k in ka_found] == [ka_key]},
    }


def _valu_mix(kname: str) -> dict:
    """The kernel's class-weighted VALU ceiling (profiles/r*_valu_mix.json, tools/valu_mix.py)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_valu_mix.json")), reverse=True):
        d = json.load(open(f)).get(kname)
        if d:
            return dict(d, source=os.path.relpath(f, REPO))
    return {}


def chip_ms_per_launch(walks: int, event_ms: float, launches: int, wall_s: float) -> float:
    """The chip's time per launch of a leg's walk kernel.  One context: the mean of the HIP events
    around its launches (what rocprofv3 reports per dispatch).  Several contexts in flight: their
    launches overlap, so an event spans its own launch and part of the others'; the chip's time per
    launch is then the timed region's wall time / all contexts' launches (host gaps included)."""
    return event_ms / launches if walks == 1 else wall_s * 1e3 / launches


def walk_roofline(kname: str, pts_launch: float, ms_launch: float, algo_bytes_per_point: float, launches: int,
                  walks: int = 1, event_ms: float | None = None, clock_mhz: float | None = None) -> dict:
    """The roofline object of one walk kernel (see the module docstring): VALU issue bound, with the
    HBM side alongside.  Counter-derived figures come from the newest profiles/r*_pmc_summary.json
    holding this kernel and are scaled to this run's points per launch.  ms_launch is the chip's time
    per launch (chip_ms_per_launch); with walks > 1 the overlapping launches' own event mean is
    reported beside it (event_mean_launch_ms, which a rocprofv3 trace of the same run agrees with).
    clock_mhz: the board's mean gfx clock over this leg's timed region, which frac_mix's ceiling uses."""
    d = pmc_entry(kname)
    secs = ms_launch / 1e3
    roof = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_GIPS, "unit": "G VALU wave-instr/s", "frac": None,
            "frac_mix": None, "traffic": None, "kernel": kname, "launches": launches, "mean_launch_ms": ms_launch,
            "walks_in_flight": walks, "event_mean_launch_ms": event_ms if event_ms is not None else ms_launch,
            "points_per_launch": pts_launch, "source": d.get("source")}
    if "valu_wave_instructions_per_dispatch" in d:
        wipp = d["valu_wave_instructions_per_dispatch"] / d["points_per_dispatch"]
        a = wipp * pts_launch / secs / 1e9
        roof.update(achieved=a, frac=a / VALU_PEAK_GIPS,
                    valu_wave_instructions_per_point=wipp, valu_lane_instructions_per_point=wipp * 64)
        if d.get("valu_issue_frac"):
            # the profiled dispatch's issue-slot occupancy at 4 cycles per instruction (clock-free)
            roof.update(pmc_valu_issue_frac_4cyc=d["valu_issue_frac"], pmc_clock_ghz=d["effective_clock_ghz"])
        for key in ("valu_dual_issue_frac", "wave_time_split", "valu_thread_cycles_per_instruction"):
            if key in d:
                roof["pmc_" + key] = d[key]
    mix = _valu_mix(kname)
    if mix.get("simd_cycles_per_point_floor"):
        # the kernel's own ceiling: its instruction mix per point at the hardware's issue floor (2 / 4
        # cycles per full- / half-rate wave64 instruction, s_nop at its in-situ cost, dual-issued
        # instructions free: tools/valu_mix.py), on every SIMD back to back, at the clock the board
        # reported over this leg (2.4 GHz if none) -- no order of these instructions issues faster
        cyc = mix["simd_cycles_per_point_floor"]
        ghz = clock_mhz / 1e3 if clock_mhz else NOMINAL_GHZ
        ceil_pts = SIMDS * ghz * 1e9 / cyc
        got_pts = pts_launch / secs
        roof.update(frac_mix=got_pts / ceil_pts, mix_floor_simd_cycles_per_point=cyc, mix_clock_ghz=ghz,
                    mix_clock_source="board gfx clock over the timed region" if clock_mhz else "nominal",
                    mix_ceiling_points_per_s=ceil_pts, mix_source=mix["source"],
                    mix_measured_cost_simd_cycles_per_point=mix.get("simd_cycles_per_point"))
        if mix.get("simd_cycles_per_point_quad"):
            # the issue model the mixed walks meet on gfx950 (one instruction per 4-cycle quad unless
            # two full-rate ones pair, tools/valu_mix.py): a model, not a bound, so no "frac"
            q = mix["simd_cycles_per_point_quad"]
            roof["quad_model"] = {"simd_cycles_per_point": q, "ceiling_points_per_s": SIMDS * ghz * 1e9 / q,
                                  "achieved_over_model": got_pts / (SIMDS * ghz * 1e9 / q)}
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


def address_leg(D: Dist, W: Walks, args, clock, mode: int, kname: str, keys_per_point: int, base0: int, ka):
    """-m rmd160 -l compress / -m xpoint: steps of C chunks of 2^32 keys from the rank's region (C / S
    per context, each in its own part of the region)."""
    import keyhunt_amd as K
    kind = K.engine.TIME_ADDRESS if mode == K.KH_MODE_ADDRESS else K.engine.TIME_XPOINT
    S = len(W)
    origin = base0 + rank_origin(D.rank, RANK_SPAN_CHUNKS) * CHUNK
    walked = 0

    def run(nc):
        nonlocal walked
        per = nc // S
        assert walked + per <= RANK_SPAN_CHUNKS // S, "rank region exhausted"

        def chunks(i, e):
            o = walk_origin(origin, i, S, RANK_SPAN_CHUNKS, CHUNK)
            for c in range(per):
                hits = e.scan(o + (walked + c) * CHUNK, CHUNK, mode, K.KH_SEARCH_COMPRESS)
                assert not hits  # the puzzle keys lie far from the start of the range
        W.each(chunks)
        walked += per

    last = 0.0
    for s in range(args.warmup_rmd):
        t = time.perf_counter()
        run(S)
        last = time.perf_counter() - t
    C = int(D.max(batch_for(args.seconds_secondary, args.steps_rmd, last / S, S, S) if args.warmup_rmd else S))
    T, t0, t1, recs, board = timed(D, W, args.steps_rmd, lambda s: run(C), C, kind, clock)
    la, ms, pts = W.kernel_time(kind)
    ka_lo, ka_n, ka_key = ka
    ka_hits = W.engs[0].scan(ka_lo, ka_n, mode, K.KH_SEARCH_COMPRESS)
    keys = D.world * args.steps_rmd * C * CHUNK * keys_per_point
    ms_launch = chip_ms_per_launch(S, ms, la, t1 - t0)
    return {"value": keys / T / 1e6, "ms_per_step": T / args.steps_rmd * 1e3, "seconds_timed": T,
            "chunks_per_step": C, "steps": args.steps_rmd,
            "points_per_s_in_kernel": pts / (ms_launch * la / 1e3),
            "roofline": walk_roofline(kname, pts / la, ms_launch, 0, la, walks=S, event_ms=ms / la,
                                      clock_mhz=(board or {}).get("board_gfxclk_mhz")),
            "sustained": quarters(t0, recs, C, CHUNK * keys_per_point, clock, board,
                                  args.steps_rmd * C * CHUNK / (recs[-1][0] - t0)),
            "known_answer": {"window": f"{ka_lo:x}:{ka_lo + ka_n - 1:x}", "expected": f"{ka_key:x}",
                             "found": [f"{h.key:x}" for h in ka_hits], "match": [h.key for h in ka_hits] == [ka_key]}}


def rmd160_leg(D: Dist, W: Walks, args, clock):
    import keyhunt_amd as K
    W.each(lambda i, e: e.set_targets([bytes.fromhex(PUZZLE66_RMD)], bloom_items=1))
    # algorithmic HBM bytes ~0 per key: the 16-B target filter block is L2-resident
    return address_leg(D, W, args, clock, K.KH_MODE_ADDRESS, "k_walk<11, 2048>", 2, 1 << 65, KA_RMD160)


def xpoint_leg(D: Dist, W: Walks, args, clock):
    """-m xpoint -f tests/63.pub -b 63 (BASELINE configs[2]): X[0..20) probes, one key per point."""
    import keyhunt_amd as K
    W.each(lambda i, e: e.set_targets([PUZZLE63_X.to_bytes(32, "big")[:20]], bloom_items=1))
    return address_leg(D, W, args, clock, K.KH_MODE_XPOINT, "k_walk<10, 2048>", 1, 1 << 62, KA_XPOINT)


def cpu_host() -> dict:
    """The host the CPU baseline ran on (lscpu): model, sockets, physical cores and threads per core,
    and the logical CPUs this process may use.  On the pool's GPU boxes a one-GPU job's CPU share is 16
    logical CPUs (OMP_NUM_THREADS, set by the box) of a much larger machine."""
    info = {"machine_cpus": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for key, name in (("Model name", "model"), ("Socket(s)", "sockets"), ("Core(s) per socket", "cores_per_socket"),
                          ("Thread(s) per core", "threads_per_core")):
            m = re.search(rf"^{re.escape(key)}:\s*(.+)$", out, re.M)
            if m:
                info[name] = m.group(1).strip()
        if str(info.get("sockets", "")).isdigit() and str(info.get("cores_per_socket", "")).isdigit():
            info["physical_cores"] = int(info["sockets"]) * int(info["cores_per_socket"])
    except Exception:
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity_cpus"] = os.cpu_count()
    tpc = info.get("threads_per_core")
    if str(tpc).isdigit() and int(tpc) > 1:
        info["job_share"] = (f"{cpu_threads()} logical CPUs = {cpu_threads() // int(tpc)} physical cores at "
                             f"{tpc} threads per core (if the share takes whole cores)")
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


# the reference CLI at its own optimisation level (oracle/Makefile.ref keyhunt_fast); the -O3 build the
# fixtures come from is the fallback
REF_BIN = next((p for p in (os.path.join(REPO, "oracle", "_ref", b) for b in ("keyhunt_fast", "keyhunt"))
                if os.path.exists(p)), os.path.join(REPO, "oracle", "_ref", "keyhunt"))
REF_FLAGS = os.path.join(REPO, "oracle", "_ref", "build_flags.txt")


def host_state(pid: int | None = None) -> dict:
    """The host's 1-min load average, the mean clock of all its CPUs and of the CPU `pid` last ran on
    (/proc): a single thread's rate follows the package's boost, which the other tenants' load sets."""
    out = {}
    try:
        out["loadavg_1min"] = os.getloadavg()[0]
        mhz = [float(l.split(":")[1]) for l in open("/proc/cpuinfo") if l.startswith("cpu MHz")]
        if mhz:
            out["cpu_mhz_mean"] = sum(mhz) / len(mhz)
        if pid:
            cpu = int(open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()[36])
            if 0 <= cpu < len(mhz):
                out["cpu_mhz_of_ref"] = mhz[cpu]
    except Exception:
        pass
    return out


def run_reference_once(argv: list[str], td: str, threads: int, seconds: float) -> tuple[int, int, dict] | None:
    """One run of the reference CLI in `td` with `threads` threads until its own stats line covers
    `seconds` (its clock starts once its tables are ready): (keys, seconds) of the last such line
    ("Total N keys in S seconds", keyhunt.cpp:2906-2946), keys counted as the reference counts them,
    and the host's state sampled every 5 s over the run (host_state, means)."""
    cmd = [REF_BIN] + argv + ["-t", str(threads), "-s", "5", "-q"]
    p = subprocess.Popen(cmd, cwd=td, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
    out = b""
    t0 = time.time()
    os.set_blocking(p.stdout.fileno(), False)
    last = None
    tick = t0
    samples, tsamp = [], t0
    while time.time() - t0 < seconds + 120:
        time.sleep(0.5)
        if time.time() - tsamp >= 5:
            tsamp = time.time()
            samples.append(host_state(p.pid))
        if time.time() - tick >= 30:
            tick = time.time()
            progress(f"CPU baseline running ({tick - t0:.0f} s, -t {threads})")
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
    state = {k: sum(x[k] for x in samples if k in x) / max(1, sum(1 for x in samples if k in x))
             for k in ("loadavg_1min", "cpu_mhz_mean", "cpu_mhz_of_ref") if any(k in x for x in samples)}
    return (last[0], last[1], state) if last and last[1] else None


def run_reference(argv: list[str], files: list[str], seconds: float, setup=None, per_core_seconds: float | None = None):
    """The reference CLI (built from /root/reference's sources by oracle/Makefile.ref) on this leg's
    workload in a scratch directory under /tmp: once with every thread of the job's CPU share (the
    baseline's value) and once with -t 1 (its per-core rate), each for `seconds` of its own stats
    clock.  `setup(dir)` may write table files first."""
    if not os.path.exists(REF_BIN):
        return None
    thr = cpu_threads()
    pcs = seconds if per_core_seconds is None else per_core_seconds
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for f in files:
            shutil.copy(os.path.join(REPO, "tests", "golden", "data", f), td)
        if setup:
            progress("CPU baseline: writing the tables for the reference")
            setup(td)
        progress(f"CPU baseline: oracle/_ref/{os.path.basename(REF_BIN)} {' '.join(argv)} -t {thr}, then -t 1")
        many = run_reference_once(argv, td, thr, seconds)
        one = run_reference_once(argv, td, 1, pcs) if pcs > 0 else None
    if not many:
        return None
    host = cpu_host()
    flags = (open(REF_FLAGS).read().strip() if os.path.exists(REF_FLAGS) and REF_BIN.endswith("_fast")
             else "oracle/_ref/keyhunt: g++ -m64 -march=x86-64-v3 -mssse3 -O3 (the fixtures' build)")
    name = f"oracle/_ref/{os.path.basename(REF_BIN)} {' '.join(argv)}"
    out = {"value": many[0] / many[1] / 1e6, "unit": "Mkeys/s", "cores": thr, "kind": "reference",
           "threads": {"value": many[0] / many[1] / 1e6, "threads": thr, "seconds": many[1], "keys": many[0],
                       "measured": True, "host_state": many[2]},
           "per_core": ({"value": one[0] / one[1] / 1e6, "threads": 1, "seconds": one[1], "keys": one[0],
                         "measured": True, "host_state": one[2]} if one else None),
           "host": host, "build_flags": flags,
           "sample": f"{name} -t {thr}: {many[0]} keys in {many[1]} s" +
                     (f"; -t 1: {one[0]} keys in {one[1]} s" if one else "") +
                     " (the reference's own stats lines, keys counted as it counts them; 'cores' = logical CPUs used)"}
    if one and host.get("physical_cores"):
        # labelled estimate, not a measurement: the -t 1 rate times the host's physical cores
        out["all_physical_cores_extrapolated"] = {"value": out["per_core"]["value"] * host["physical_cores"],
                                                  "cores": host["physical_cores"], "measured": False}
    return out


def cpu_baseline_bsgs(eng, C: dict, seconds: float, per_core_seconds: float | None = None):
    """The reference's BSGS giant-step loop (thread_process_bsgs, keyhunt.cpp:4549-4888) on the host,
    on the same workload (-b bits -k K from 2^(bits-1)).  Its 120-s-per-core baby-step build is
    skipped: the engine writes the four -S table files (kh_bsgs_save: the reference's format, byte
    for byte, tests/test_gpu_tables.py) and the reference reads them (-S -6, keyhunt.cpp:1983-2240)."""
    pub = {125: "125.txt", 130: "130.txt"}[C["bits"]]
    return run_reference(["-m", "bsgs", "-f", pub, "-b", str(C["bits"]), "-k", str(C["k"]), "-S", "-6"], [pub],
                         seconds, setup=lambda d: eng.bsgs_save(d), per_core_seconds=per_core_seconds)


def cpu_baseline_rmd160(seconds: float, per_core_seconds: float | None = None):
    return run_reference(["-m", "rmd160", "-f", "66.rmd", "-b", "66", "-l", "compress"], ["66.rmd"], seconds,
                         per_core_seconds=per_core_seconds)


def cpu_baseline_xpoint(seconds: float, per_core_seconds: float | None = None):
    return run_reference(["-m", "xpoint", "-f", "63.pub", "-b", "63"], ["63.pub"], seconds,
                         per_core_seconds=per_core_seconds)


def legs_summary(line: dict) -> dict:
    """The three legs in a few hundred bytes, for the end of the line: value, unit, the known-answer
    match, the dominant kernel's roofline frac and the CPU baseline (value, threads, seconds)."""
    out = {}
    for name, leg in (("bsgs_b125" if "b 125" in line["config"]["workload"] else "bsgs_b130", line),
                      ("rmd160_b66", line.get("secondary")), ("xpoint_b63", line.get("tertiary"))):
        if not leg:
            continue
        cb = leg.get("cpu_baseline") or {}
        th = cb.get("threads") or {}
        out[name] = {"value": leg["value"], "unit": leg["unit"], "known_answer_match": leg["known_answer"]["match"],
                     "frac": (leg.get("roofline") or {}).get("frac"),
                     "cpu_baseline": {"value": cb.get("value"), "threads": th.get("threads"), "seconds": th.get("seconds"),
                                      "per_core_seconds": (cb.get("per_core") or {}).get("seconds")} if cb else None}
    return out


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
    ap.add_argument("--bases", type=int, default=0,
                    help="BSGS bases per warm-up step per GPU, and the quantum of the timed steps' batch (0: per config)")
    ap.add_argument("--seconds", type=float, default=60.0,
                    help="size the BSGS batch so that the timed steps last this long (0: --bases per step)")
    ap.add_argument("--seconds-secondary", type=float, default=20.0,
                    help="the same for each address-family leg (0: one 2^32-key chunk per step)")
    ap.add_argument("--steps-rmd", type=int, default=None)
    ap.add_argument("--warmup-rmd", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="CPU baseline of the rmd160 / xpoint legs: seconds of the reference's own stats clock on the "
                         "job's threads (>= 60 s of steady state, SURVEY.md 8d)")
    ap.add_argument("--cpu-seconds-primary", type=float, default=60.0,
                    help="the same for the BSGS leg (the line's cpu_baseline)")
    ap.add_argument("--cpu-seconds-per-core", type=float, default=30.0,
                    help="every leg's -t 1 run (the per-core rate beside the baseline's value)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="only the CPU baselines of the three legs (the BSGS one still needs the GPU to write the "
                         "-S tables); prints one JSON object")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--rehearse", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share devices; the line reports it)")
    ap.add_argument("--walks", type=int, default=WALKS_BSGS, choices=(1, 2, 4),
                    help="BSGS leg: contexts per GPU, each on its own stream and host thread (walk launches in flight)")
    ap.add_argument("--walks-secondary", type=int, default=WALKS_ADDRESS, choices=(1, 2, 4),
                    help="the same for the rmd160 and xpoint legs")
    ap.add_argument("--layer1", type=int, default=1, help="BSGS layer-1 layout: 1 blocked (default), 0 reference")
    args = ap.parse_args()
    args.steps_rmd = args.steps if args.steps_rmd is None else args.steps_rmd
    args.warmup_rmd = args.warmup if args.warmup_rmd is None else args.warmup_rmd

    import keyhunt_amd as K
    D = Dist()
    if args.gpus != D.world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={D.world}: launch one rank per GPU")
    dev = device_plan(D.world, D.local, D.local_world, K.device_count(), args.rehearse)
    W = Walks(K, dev, max(args.walks, 1 if args.no_secondary else args.walks_secondary))
    bdf = pci_bus_id(dev)
    clock = BoardSampler(bdf).start()
    if args.cpu_only:  # the reference's rates alone (profiles/r04*_cpu_baseline_*.json)
        C = BSGS_CONFIGS[args.config]
        W.engs[0].bsgs_setup(1 << 44, C["k"], layer1=args.layer1)
        W.engs[0].bsgs_build()
        pc = args.cpu_seconds_per_core
        res = {"bsgs": cpu_baseline_bsgs(W.engs[0], C, args.cpu_seconds, pc),
               "rmd160": cpu_baseline_rmd160(args.cpu_seconds, pc), "xpoint": cpu_baseline_xpoint(args.cpu_seconds, pc),
               "cpu_seconds": args.cpu_seconds, "workload": C["workload"]}
        W.close()
        json_out.write(json.dumps(res) + "\n")
        json_out.flush()
        return
    prim = bsgs_leg(D, W.head(args.walks), args, clock)
    Wa = W.head(args.walks_secondary)
    sec = None if args.no_secondary else rmd160_leg(D, Wa, args, clock)
    ter = None if args.no_secondary else xpoint_leg(D, Wa, args, clock)
    clock.stop()
    cpu_b = cpu_r = cpu_x = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu_baseline and not args.cpu_only:
        pc = args.cpu_seconds_per_core
        cpu_b = cpu_baseline_bsgs(W.engs[0], BSGS_CONFIGS[args.config], args.cpu_seconds_primary, pc)
        if not args.no_secondary:
            cpu_r = cpu_baseline_rmd160(args.cpu_seconds, pc)
            cpu_x = cpu_baseline_xpoint(args.cpu_seconds, pc)
    W.close()
    ranks = D.gather({"rank": D.rank, "host": os.uname().nodename, "device": dev, "pci_bus_id": bdf,
                      "giant_points_per_s": prim["rank_giant_points_per_s"]})
    kas = [prim["known_answer"]] + [x["known_answer"] for x in (sec, ter) if x]
    ka_ok = D.sum(float(all(k["match"] for k in kas))) == D.world
    D.barrier()
    if D.rank == 0:
        info = prim["info"]
        devices = sorted({(r["host"], r["pci_bus_id"] or f"hip{r['device']}") for r in ranks})
        line = {
            "metric": METRIC, "value": prim["value"], "unit": "Mkeys/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": prim["ms_per_step"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32",
            "data": f"synthetic: {BSGS_CONFIGS[args.config]['data']}, sequential bases from 2^{BSGS_CONFIGS[args.config]['bits'] - 1}",
            "config": {"workload": BSGS_CONFIGS[args.config]["workload"], "n": info.n, "k": BSGS_CONFIGS[args.config]["k"], "m": info.m,
                       "layer1_layout": "blocked" if info.layer1_layout == 1 else "reference",
                       "bases_per_step": prim["bases_per_step"],
                       "giant_points_per_step": prim["bases_per_step"] * info.cycles * 1024,
                       "walks_in_flight_per_gpu": args.walks,
                       "placement_calibration": prim["placement_calibration"],
                       "parallelism": f"keyspace split x{D.world} (no collective)"},
            "devices_used": len(devices),
            "rehearsal": len(devices) < D.world,
            "ranks": ranks,
            "seconds_timed": prim["seconds_timed"],
            "giant_points_per_s": prim["giant_points_per_s"],
            "build_seconds": prim["build_seconds"],
            "first_level_candidates": prim["candidates"],
            "known_answer": prim["known_answer"],
            "known_answers_all_ranks_match": ka_ok,
            "sustained": prim["sustained"],
            "roofline": prim["roofline"],
            "random_access": prim["random_access"],
            "board_sampler": dict(clock.info(), source="amdsmi gpu_metrics / energy counter of the rank-0 device"),
            "cpu_baseline": cpu_b,
        }
        for key, leg, wl in (("secondary", sec, "-m rmd160 -f tests/66.rmd -b 66 -l compress"),
                             ("tertiary", ter, "-m xpoint -f tests/63.pub -b 63")):
            if leg:
                line[key] = {"workload": wl, "value": leg["value"], "walks_in_flight_per_gpu": args.walks_secondary, "unit": "Mkeys/s", "ms_per_step": leg["ms_per_step"],
                             "steps": leg["steps"], "chunks_per_step": leg["chunks_per_step"],
                             "seconds_timed": leg["seconds_timed"],
                             "points_per_s_in_kernel": leg["points_per_s_in_kernel"],
                             "known_answer": leg["known_answer"], "sustained": leg["sustained"],
                             "roofline": leg["roofline"],
                             "cpu_baseline": cpu_r if key == "secondary" else cpu_x}
        line["legs"] = legs_summary(line)
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    D.close()
    if not ka_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
