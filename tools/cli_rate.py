#!/usr/bin/env python3
"""Sustained rate of the CLI (bin/keyhunt-amd) as a user sees it, beside bench.py's line.

Runs the CLI on one workload for --seconds from a scratch copy of tests/golden/data with its stats
line every 5 s, and timestamps every stats line on the host as it arrives.  Reports, per stats line,
the CLI's own cumulative figure ("Total N keys in S seconds", keyhunt.cpp:2906-2946) and the host
clock, and the steady rate between the first line after --skip seconds and the last line computed two
ways: from the CLI's own seconds and from the host clock.  The CLI's seconds count its stats loop's
sleep(1) ticks, so they drift behind the host clock (each tick is 1 s plus the loop's own work): the
host-clock rate is the engine's delivered rate, the CLI-seconds rate what its stats line shows.

usage: python tools/cli_rate.py --mode bsgs|rmd160|xpoint [--seconds 70] [--skip 20] [--out FILE]
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "keyhunt_amd", "bin", "keyhunt-amd")
ARGV = {"bsgs": ["-m", "bsgs", "-f", "125.txt", "-b", "125", "-k", "128"],
        "rmd160": ["-m", "rmd160", "-f", "66.rmd", "-b", "66", "-l", "compress"],
        "xpoint": ["-m", "xpoint", "-f", "63.pub", "-b", "63"],
        # -R: every chunk starts at a random key, so every call sets its 2^20 lanes up again
        "xpoint_random": ["-m", "xpoint", "-f", "63.pub", "-b", "63", "-R"],
        "rmd160_random": ["-m", "rmd160", "-f", "66.rmd", "-b", "66", "-l", "compress", "-R"],
        # BSGS base schedules other than sequential go through kh_bsgs_scan_list (lanes restart per call)
        "bsgs_random": ["-m", "bsgs", "-f", "125.txt", "-b", "125", "-k", "128", "-B", "random"],
        "bsgs_both": ["-m", "bsgs", "-f", "125.txt", "-b", "125", "-k", "128", "-B", "both"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=sorted(ARGV), required=True)
    ap.add_argument("--seconds", type=float, default=70)
    ap.add_argument("--skip", type=float, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    td = tempfile.mkdtemp()
    for fn in os.listdir(os.path.join(REPO, "tests", "golden", "data")):
        shutil.copy(os.path.join(REPO, "tests", "golden", "data", fn), td)
    argv = [CLI] + ARGV[a.mode] + ["-s", "5", "-q"]
    t0 = time.time()
    p = subprocess.Popen(argv, cwd=td, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
    os.set_blocking(p.stdout.fileno(), False)
    buf, lines = b"", []
    while time.time() - t0 < a.seconds and p.poll() is None:
        time.sleep(0.05)
        try:
            c = p.stdout.read()
        except Exception:
            c = None
        if c:
            buf += c
            for m in re.finditer(rb"Total (\d+) keys in (\d+) seconds", buf):
                lines.append({"host_s": round(time.time() - t0, 3), "keys": int(m.group(1)), "cli_s": int(m.group(2))})
            buf = buf[buf.rfind(b"seconds") + 7:] if b"seconds" in buf else buf
    p.terminate()
    try:
        p.wait(timeout=20)
    except subprocess.TimeoutExpired:
        p.kill()
    shutil.rmtree(td, ignore_errors=True)
    steady = [x for x in lines if x["host_s"] >= a.skip]
    res = {"mode": a.mode, "argv": argv[1:], "lines": lines}
    if len(steady) >= 2:
        f, l = steady[0], steady[-1]
        dk = l["keys"] - f["keys"]
        res["steady"] = {"from_host_s": f["host_s"], "to_host_s": l["host_s"],
                         "keys_per_s_cli_seconds": dk / max(1, l["cli_s"] - f["cli_s"]),
                         "keys_per_s_host_clock": dk / (l["host_s"] - f["host_s"]),
                         "cli_seconds_per_host_second": (l["cli_s"] - f["cli_s"]) / (l["host_s"] - f["host_s"])}
    s = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    sys.exit(main())
