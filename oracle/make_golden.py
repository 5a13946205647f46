#!/usr/bin/env python3
"""Regenerate the committed golden fixtures from the REFERENCE built by oracle/Makefile.ref.

TEST INFRASTRUCTURE.  Runs in the development container only (needs /root/reference):

  tests/golden/ref_vectors.json  primitive vectors printed by oracle/_ref/ref_golden (field ops,
                                 pubkeys, hash160 02/03/04, XXH64, bloom sizing/fill, group
                                 walk, BSGS baby tables at small M)
  tests/golden/ref_e2e.json      end-to-end hit sets of oracle/_ref/keyhunt (the reference CLI) on
                                 known-answer windows, parsed from the
                                 KEYFOUNDKEYFOUND.txt it writes.
  tests/golden/ref_tables.json   digests of the -S table files the reference CLI writes at small
                                 (n, k) (heap pointers masked).
  tests/golden/ref_data/         the -S target caches (data_<hex>.dat) the reference CLI writes for
                                 address / rmd160 / xpoint / eth target files, with
                                 ref_data/index.json (name, size, masked sha256, hit set of the run).
  tests/golden/ref_mapped.json   --mapped bloom files the reference CLI leaves after run sequences
                                 (fresh, reload, chunks, size overrides, --create-mapped/--load-bloom,
                                 BSGS shard files), with the hit sets of the runs.
  tests/golden/ref_bsgsd.json    a transcript of the reference daemon (oracle/_ref/bsgsd): every
                                 request of BSGSD_REQUESTS with the raw reply bytes and the lines the
                                 daemon printed for it, plus its KEYFOUNDKEYFOUND.txt.

  tests/golden/ref_stdout.json   the reference CLI's whole stdout of single-thread runs with -M and
                                 without -q (progress lines), and its stats lines with and without -M.

Usage:  python oracle/make_golden.py [--vectors] [--e2e] [--tables] [--data] [--bsgsd] [--stdout]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DATA = os.path.join(REPO, "tests", "golden", "data")
REF_BIN = os.path.join(HERE, "_ref", "keyhunt")
REF_GOLDEN = os.path.join(HERE, "_ref", "ref_golden")

# (name, argv after the binary, timeout s).  Windows from SURVEY.md 8c.
E2E_RUNS = [
    ("address_1to32_2p20", ["-m", "address", "-f", "1to32.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    # malformed lines among the targets (tests/golden/make_ragged_targets.py): the reference's
    # line counting and reading order decide which targets are loaded; stderr lines recorded
    ("ragged_address_2p20", ["-m", "address", "-f", "ragged_addr.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("ragged_rmd160_2p20", ["-m", "rmd160", "-f", "ragged_addr.txt", "-l", "compress", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("ragged_xpoint_2p20", ["-m", "xpoint", "-f", "ragged_x.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    # keys within 2^20 of the group order (tests/golden/make_near_order_targets.py)
    ("address_near_order", ["-m", "address", "-f", "near_order_addr.txt", "-l", "compress", "-r",
                            "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0264141:fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364140",
                            "-n", "0x100000", "-t", "8"], 300),
    ("xpoint_near_order", ["-m", "xpoint", "-f", "near_order_x.txt", "-r",
                           "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0264141:fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364140",
                           "-n", "0x100000", "-t", "8"], 300),
    ("ragged_bsgs_63_window", ["-m", "bsgs", "-f", "ragged_bsgs.txt", "-r", "7cce5a0000000000:7cce9a0000000000", "-t", "8"], 300),
    ("ragged_bsgs_bad_digit", ["-m", "bsgs", "-f", "ragged_bsgs_bad.txt", "-r", "7cce5a0000000000:7cce9a0000000000", "-t", "8"], 60),
    ("rmd160_1to32_compress_2p20", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("xpoint_1to63_65_2p20", ["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_66_window", ["-m", "rmd160", "-f", "66.rmd", "-l", "compress", "-r", "2832ed74f2b000000:2832ed74f2bffffff", "-n", "0x100000", "-t", "8"], 600),
    ("address_66_window", ["-m", "address", "-f", "66.txt", "-l", "compress", "-r", "2832ed74f2b400000:2832ed74f2b7fffff", "-n", "0x100000", "-t", "8"], 600),
    ("rmd160_64_window", ["-m", "rmd160", "-f", "64.rmd", "-l", "compress", "-r", "f7051f27b0000000:f7051f27b0ffffff", "-n", "0x100000", "-t", "8"], 600),
    ("xpoint_63_window", ["-m", "xpoint", "-f", "63.pub", "-r", "7cce5efdac000000:7cce5efdacffffff", "-n", "0x100000", "-t", "8"], 600),
    # -e (endomorphism: (beta*X, Y) and (beta^2*X, Y) checked too, keyhunt.cpp:3408-3830)
    ("address_1to32_2p20_endo", ["-m", "address", "-f", "1to32.txt", "-r", "1:100000", "-n", "0x100000", "-e", "-t", "8"], 300),
    ("rmd160_1to32_compress_2p20_endo", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:100000", "-n", "0x100000", "-e", "-t", "8"], 300),
    ("xpoint_1to63_65_2p20_endo", ["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:100000", "-n", "0x100000", "-e", "-t", "8"], 300),
    # targets built from lambda-multiples of small keys (tests/golden/make_endo_targets.py)
    ("address_endo_targets", ["-m", "address", "-f", "endo_addr.txt", "-r", "1:100000", "-n", "0x100000", "-e", "-t", "8"], 300),
    ("address_endo_targets_no_e", ["-m", "address", "-f", "endo_addr.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("xpoint_endo_targets", ["-m", "xpoint", "-f", "endo_x.txt", "-r", "1:100000", "-n", "0x100000", "-e", "-t", "8"], 300),
    # -c eth: Keccak-256(X||Y)[12:32] targets (tests/golden/make_eth_targets.py)
    ("address_eth_2p20", ["-m", "address", "-c", "eth", "-f", "eth_targets.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_eth_2p20", ["-m", "rmd160", "-c", "eth", "-f", "eth_targets.rmd", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    # -m vanity: base58 prefixes -> hash160 ranges (keyhunt.cpp:6739-6866), VANITYKEYFOUND.txt
    ("vanity_2p20_compress", ["-m", "vanity", "-v", "1Kha", "-v", "1PUB", "-l", "compress", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("vanity_2p20_both", ["-m", "vanity", "-v", "1Kha", "-v", "1PUB", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("vanity_2p20_uncompress_endo", ["-m", "vanity", "-v", "1Kha", "-v", "1PUB", "-l", "uncompress", "-e", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("vanity_2p20_compress_endo", ["-m", "vanity", "-v", "1Kha", "-v", "1PUB", "-l", "compress", "-e", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("vanity_file_2p20", ["-m", "vanity", "-f", "vanity.txt", "-l", "compress", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("bsgs_120_window", ["-m", "bsgs", "-f", "120.txt", "-r", "b10f22572c497a836e9d0000000000:b10f22572c497a836edd0000000000", "-t", "8"], 300),
    ("bsgs_125_window", ["-m", "bsgs", "-f", "125.txt", "-r", "1c533b6bb7f0804e0995fe0000000000:1c533b6bb7f0804e09963e0000000000", "-t", "8"], 300),
    ("bsgs_130_window", ["-m", "bsgs", "-f", "130.txt", "-r", "33e7665705359f04f28b8880000000000:33e7665705359f04f28b8c80000000000", "-t", "8"], 300),
    ("bsgs_63_window", ["-m", "bsgs", "-f", "63.pub", "-r", "7cce5a0000000000:7cce9a0000000000", "-t", "8"], 300),
    ("bsgs_test120_b120", ["-m", "bsgs", "-f", "test120.txt", "-b", "120", "-t", "8"], 300),
    ("bsgs_63_small_n_k4", ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "4", "-r", "7cce5efdac000000:7cce5efdad000000", "-t", "8"], 300),
    # non-power-of-two k: bases overlap (cycles*1024 > aux, SURVEY.md 8a parity note 13)
    ("bsgs_63_k20", ["-m", "bsgs", "-f", "63.pub", "-k", "20", "-r", "7cce5a0000000000:7cce9a0000000000", "-t", "8"], 300),
    ("bsgs_63_small_n_k3", ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "3", "-r", "7cce5efdac000000:7cce5efdad000000", "-t", "8"], 300),
    # deterministic base schedules (keyhunt.cpp:5953 backward, 6211 both)
    ("bsgs_63_backward", ["-m", "bsgs", "-f", "63.pub", "-B", "backward", "-r", "7cce5a0000000000:7cce9a0000000000", "-t", "8"], 300),
    ("bsgs_63_both", ["-m", "bsgs", "-f", "63.pub", "-B", "both", "-r", "7cce5a0000000000:7cce9a0000000000", "-t", "8"], 300),
    # GGSB: bases every 2 x block size (keyhunt.cpp:1477-1499, 1617-1627), sequential worker
    ("bsgs_63_ggsb_count4", ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "4", "-B", "ggsb", "--bsgs-block-count", "4", "-r", "7cce5efdac000000:7cce5efdad000000", "-t", "8"], 300),
    ("bsgs_63_ggsb_size1024_both", ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "4", "-B", "both", "--bsgs-block-size", "1024", "-r", "7cce5efdac000000:7cce5efdad000000", "-t", "8"], 300),
    # -e -c eth: the six eth images per point, with the reference's repeated beta image
    # (keyhunt.cpp:3524-3536, 3703-3760; tests/golden/make_eth_endo_targets.py)
    ("address_eth_endo_2p20", ["-m", "address", "-c", "eth", "-e", "-f", "eth_endo.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    ("address_eth_2p20_endo", ["-m", "address", "-c", "eth", "-e", "-f", "eth_targets.txt", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    # one thread, so the file's record order is the reference's per-point slot order (ORDERED)
    ("address_eth_endo_pair_t1", ["-m", "address", "-c", "eth", "-e", "-f", "eth_endo_pair.txt", "-r", "1:100000", "-n", "0x100000", "-t", "1"], 300),
    # -r START without END runs to the group order (keyhunt.cpp:1028-1033): BSGS ends at "All points
    # were found"; the address family never ends, so it is stopped after `tmo` s and only hits
    # below the "cmp_below" key are compared
    ("bsgs_63_start_only", ["-m", "bsgs", "-f", "63.pub", "-r", "7cce5a0000000000", "-t", "8"], 300),
    ("xpoint_63_start_only", ["-m", "xpoint", "-f", "63.pub", "-r", "7cce5efdac000000", "-n", "0x100000", "-t", "8"], 20),
    # a key exactly at a base start: keyhunt's worker reaches it only through the point at infinity
    # and misses it (bsgsd has an extra per-base test and finds it, tests/golden/ref_bsgsd.json)
    ("bsgs_63_key_at_base", ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "2", "-r", "7cce5efdaccf6808:7cce5efdadcf6808", "-t", "8"], 300),
    # --rmd-batch-size below 1024 (keyhunt.cpp:815-829, 3301-3461): groups of G whose batch
    # inversion returns 0, so only each group's centre is a real point (targets from
    # tests/golden/make_rmd_batch_targets.py); 1001 rounds down to 1000, eth walks the same points
    ("rmd160_batch512_compress", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "compress", "--rmd-batch-size", "512", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_batch512_both", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "both", "--rmd-batch-size", "512", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_batch512_both_endo", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "both", "-e", "--rmd-batch-size", "512", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_batch1000_compress", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "compress", "--rmd-batch-size", "1000", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_batch1000_both", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "both", "--rmd-batch-size", "1000", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_batch1001_compress_endo", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "compress", "-e", "--rmd-batch-size", "1001", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_batch1024_both", ["-m", "rmd160", "-f", "rmd_batch.rmd", "-l", "both", "--rmd-batch-size", "1024", "-r", "10000:20ffff", "-n", "0x100000", "-t", "8"], 300),
    ("rmd160_eth_batch8", ["-m", "rmd160", "-c", "eth", "-f", "eth_targets.rmd", "--rmd-batch-size", "8", "-r", "1:100000", "-n", "0x100000", "-t", "8"], 300),
    # no range at all: sequential from 1 (keyhunt.cpp:1250-1255)
    ("address_1to32_no_range", ["-m", "address", "-f", "1to32.txt", "-l", "compress", "-n", "0x100000", "-t", "8"], 20),
]
# stopped runs: compare the hits with keys below this bound
CMP_BELOW = {"xpoint_63_start_only": 0x7cce5efdad000000, "address_1to32_no_range": 1 << 24}

# the hit blocks the reference prints on stdout (writekey 6914, writekeyeth 6946, writevanitykey
# 6728) and the two BSGS lines, taken apart because the reference's threads may interleave them
# (the sequential worker's first line has no newline, 4826-4827; random 5079, dance 5885,
# backward 6144 and both 6429 end it with one)
STDOUT_BLOCK = re.compile(r"\nHit! Private Key: [^\n]*\npubkey: [^\n]*\nAddress [^\n]*\nrmd160 [^\n]*\n"
                          r"|\n Hit!!!! Private Key: [^\n]*\naddress: [^\n]*\n"
                          r"|\nVanity Private Key: [^\n]*\npubkey: [^\n]*\nAddress [^\n]*\nrmd160 [^\n]*\n"
                          r"|\[\+\] Thread Key found privkey [0-9a-f]+ *\n?|\[\+\] Publickey [^\n]*\n")


def stdout_blocks(text: str) -> list[str]:
    return sorted(STDOUT_BLOCK.findall(text))


# -S table files (keyhunt.cpp:2504-2652) written by the reference for small (n, k): their sha256
# with each struct bloom's `bf` heap pointer (bytes 64..72 of every 112-byte header) zeroed
TABLE_RUNS = [
    ("n1000000_k2", ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "2", "-r", "7cce5efdac000000:7cce5efdad000000", "-S", "-t", "4"]),
    ("n4000000_k3", ["-m", "bsgs", "-f", "63.pub", "-n", "0x4000000", "-k", "3", "-r", "7cce5efdac000000:7cce5efdb0000000", "-S", "-t", "4"]),
    # layer 1 past the 10000-entry floor (M/256 = 16384 entries per shard)
    ("n100000000_k64", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000000", "-k", "64", "-r", "7cce5efd00000000:7cce5efe00000000", "-S", "-t", "8"]),
]


def masked_table_digest(path: str) -> str:
    import hashlib
    data = bytearray(open(path, "rb").read())
    if path.endswith(".blm"):
        rec = len(data) // 256
        for i in range(256):
            data[i * rec + 64: i * rec + 72] = bytes(8)
    return hashlib.sha256(bytes(data)).hexdigest()


def gen_tables() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    out = {}
    for name, argv in TABLE_RUNS:
        with tempfile.TemporaryDirectory() as td:
            shutil.copy(os.path.join(DATA, "63.pub"), td)
            p = subprocess.run(["timeout", "300", REF_BIN] + argv + ["-q"], cwd=td, capture_output=True, text=True)
            files = sorted(f for f in os.listdir(td) if f.startswith("keyhunt_bsgs_"))
            out[name] = {"argv": argv, "exit": p.returncode,
                         "files": {f: masked_table_digest(os.path.join(td, f)) for f in files},
                         "sizes": {f: os.path.getsize(os.path.join(td, f)) for f in files}}
            print(name, p.returncode, files, flush=True)
    out["_generator"] = "oracle/make_golden.py --tables: oracle/_ref/keyhunt -S (reference CLI built from its sources)"
    with open(os.path.join(REPO, "tests", "golden", "ref_tables.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


# -S target caches (keyhunt.cpp:7756-7855): data_<hex>.dat per target file
DATA_RUNS = [
    ("address_1to32", "1to32.txt", ["-m", "address", "-f", "1to32.txt", "-r", "1:FFFFF", "-n", "0x100000", "-S", "-t", "2"]),
    ("rmd160_1to32", "1to32.rmd", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:FFFFF", "-n", "0x100000", "-S", "-t", "2"]),
    ("xpoint_1to63_65", "1to63_65.txt", ["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:FFFFF", "-n", "0x100000", "-S", "-t", "2"]),
    ("eth_targets", "eth_targets.txt", ["-m", "address", "-c", "eth", "-f", "eth_targets.txt", "-r", "1:FFFFF", "-n", "0x100000", "-S", "-t", "2"]),
    # > 10000 rows with -z 2: bloom entries = 2 x items (keyhunt.cpp:7608); the 330 KB cache itself
    # is not committed, only its digest (the target file comes from tests/golden/make_many_targets.py)
    ("rmd160_many_z2", "many.rmd", ["-m", "rmd160", "-f", "many.rmd", "-l", "compress", "-r", "1:FFFFF", "-n", "0x100000", "-z", "2", "-S", "-t", "2"]),
]


def masked_data_digest(path: str) -> str:
    """sha256 of a data_<hex>.dat with the struct bloom's `bf` heap pointer (file bytes 96..104) zeroed."""
    import hashlib
    data = bytearray(open(path, "rb").read())
    data[32 + 64: 32 + 72] = bytes(8)
    return hashlib.sha256(bytes(data)).hexdigest()


def gen_data() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    dst = os.path.join(REPO, "tests", "golden", "ref_data")
    os.makedirs(dst, exist_ok=True)
    index = {}
    for name, src, argv in DATA_RUNS:
        with tempfile.TemporaryDirectory() as td:
            if src == "many.rmd":
                import sys
                sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
                import make_many_targets
                make_many_targets.write(os.path.join(td, src))
            else:
                shutil.copy(os.path.join(DATA, src), td)
            p = subprocess.run(["timeout", "120", REF_BIN] + argv + ["-q"], cwd=td, capture_output=True, text=True)
            files = [f for f in os.listdir(td) if f.startswith("data_")]
            assert len(files) == 1, (name, files, p.stdout, p.stderr)
            f = files[0]
            if src != "many.rmd":
                shutil.copy(os.path.join(td, f), os.path.join(dst, f))
            kf = os.path.join(td, "KEYFOUNDKEYFOUND.txt")
            hits = parse_keyfound(open(kf).read()) if os.path.exists(kf) else []
            index[name] = {"argv": argv, "source": src, "file": f, "size": os.path.getsize(os.path.join(td, f)),
                           "masked_sha256": masked_data_digest(os.path.join(td, f)),
                           "keys": sorted({h["key"] for h in hits}), "committed": src != "many.rmd"}
            print(name, p.returncode, f, flush=True)
    index["_generator"] = "oracle/make_golden.py --data: oracle/_ref/keyhunt -S (reference CLI built from its sources)"
    with open(os.path.join(dst, "index.json"), "w") as fh:
        json.dump(index, fh, indent=1, sort_keys=True)


def gen_vectors() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    out = subprocess.run([REF_GOLDEN], check=True, capture_output=True, text=True).stdout
    doc = json.loads(out)
    doc["_generator"] = "oracle/_ref/ref_golden (oracle/ref_golden.cpp linked against the reference's own sources)"
    with open(os.path.join(REPO, "tests", "golden", "ref_vectors.json"), "w") as f:
        json.dump(doc, f, indent=1)


def parse_keyfound(text: str) -> list[dict]:
    hits = []
    for m in re.finditer(r"(Vanity )?Private Key: ([0-9a-f]+)\npubkey: ([0-9a-f]+)\nAddress (\S+)\nrmd160 ([0-9a-f]+)", text):
        h = {"key": m.group(2), "pubkey": m.group(3), "address": m.group(4), "rmd160": m.group(5)}
        if m.group(1):
            h["vanity"] = True
        hits.append(h)
    for m in re.finditer(r"Key found privkey ([0-9a-f]+)\nPublickey ([0-9a-f]+)", text):
        hits.append({"key": m.group(1), "pubkey": m.group(2)})
    for m in re.finditer(r"Private Key: ([0-9a-f]+)\naddress: (0x[0-9a-f]+)\n", text):  # writekeyeth
        hits.append({"key": m.group(1), "address": m.group(2)})
    return hits


# the reference's notes on target-file lines it skips (keyhunt.cpp:7299, 7433, 7468, 7479)
STDERR_NOTE = re.compile(r"^\[[IE]\] (?:Ommiting|Omiting|Ignoring)[^\n]*$", re.M)
# and on public keys it refuses (keyhunt.cpp:1433; SECP256K1.cpp:303-380)
STDOUT_NOTE = re.compile(r"^(?:ParsePublicKeyHex: |Invalid length: )[^\n]*$", re.M)


# single-thread runs whose KEYFOUNDKEYFOUND.txt record order is pinned too ("hits_in_order")
ORDERED = {"address_eth_endo_pair_t1"}


def gen_e2e(only: list[str] | None = None) -> None:
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    path = os.path.join(REPO, "tests", "golden", "ref_e2e.json")
    results = json.load(open(path)) if os.path.exists(path) else {}
    for name, argv, tmo in E2E_RUNS:
        if only and name not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            for fn in os.listdir(DATA):
                shutil.copy(os.path.join(DATA, fn), td)
            p = subprocess.run(["timeout", str(tmo), REF_BIN] + argv + ["-q"], cwd=td, capture_output=True, text=True)
            text = ""
            for fn in ("KEYFOUNDKEYFOUND.txt", "VANITYKEYFOUND.txt"):
                kf = os.path.join(td, fn)
                text += open(kf).read() if os.path.exists(kf) else ""
            hits = sorted(parse_keyfound(text), key=lambda h: int(h["key"], 16))
            blocks = stdout_blocks(p.stdout)
            results[name] = {"argv": argv, "exit": p.returncode, "hits": hits, "stdout_blocks": blocks}
            if name in ORDERED:
                results[name]["hits_in_order"] = parse_keyfound(text)
            if name.startswith("ragged"):
                results[name]["stderr_lines"] = STDERR_NOTE.findall(p.stderr)
                results[name]["stdout_notes"] = STDOUT_NOTE.findall(p.stdout)
            if name in CMP_BELOW:
                lim = CMP_BELOW[name]
                results[name].update(cmp_below=hex(lim), killed_after=tmo,
                                     hits=[h for h in hits if int(h["key"], 16) < lim],
                                     stdout_blocks=[b for b in blocks if int(re.search(r"Key: ([0-9a-f]+)", b).group(1), 16) < lim])
            print(f"{name}: exit={p.returncode} hits={len(hits)}", flush=True)
    results["_generator"] = "oracle/make_golden.py running oracle/_ref/keyhunt (reference CLI built from its sources)"
    with open(path, "w") as f:
        json.dump(results, f, indent=1, sort_keys=True)


PUB63 = "0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579"


def http_post(body: str) -> bytes:
    b = body.encode()
    return (b"POST / HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"
            % len(b)) + b


# (name, raw request bytes) for the daemon transcript (bsgsd.cpp:3307-3579): found (both range
# spellings, and a key at the very start of a base, bsgsd.cpp:2544-2561), not found, malformed
# lines, a bad pubkey prefix / length, and the HTTP POST forms
BSGSD_REQUESTS = [
    ("line_found", f"{PUB63} 7cce5efdac000000:7cce5efdad000000\n".encode()),
    ("line_found_3tok", f"{PUB63} 7cce5efdac000000 7cce5efdad000000\n".encode()),
    ("line_found_at_base", f"{PUB63} 7cce5efdaccf6808:7cce5efdadcf6808\n".encode()),
    ("line_not_found", f"{PUB63} 4000000000000000:4000000001000000\n".encode()),
    ("line_one_token", b"nonsense\n"),
    ("line_no_colon", f"{PUB63} 7cce5efdac000000\n".encode()),
    ("line_bad_hex", f"{PUB63} zz:7cce5efdad000000\n".encode()),
    ("line_bad_prefix", b"0565ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579 1:2\n"),
    ("line_short_02", b"0265ec2994b8 1:2\n"),
    ("http_found", http_post(json.dumps({"pubkey": PUB63, "from": "7cce5efdac000000", "to": "7cce5efdad000000"}))),
    ("http_not_found", http_post(json.dumps({"pubkey": PUB63, "from": "4000000000000000", "to": "4000000001000000"}))),
    ("http_missing_field", http_post(json.dumps({"pubkey": PUB63}))),
    ("http_bad_hex", http_post(json.dumps({"pubkey": PUB63, "from": "xyz", "to": "7cce5efdad000000"}))),
]
BSGSD_ARGS = ["-n", "0x1000000", "-k", "2"]


def mask_elapsed(reply: bytes) -> bytes:
    return re.sub(rb"X-Elapsed-Seconds: [0-9.]+", b"X-Elapsed-Seconds: *", reply)


# daemon starts whose table files are recorded: (name, extra args, fresh directory?)
BSGSD_STARTS = [
    ("default", [], True),
    ("default_restart", [], False),
    ("ptable_cache", ["--ptable", "pt.bin", "--ptable-cache"], True),
    ("ptable_load_cache", ["--ptable", "pt.bin", "--load-ptable", "--ptable-cache"], False),
]


def start_ref_daemon(cwd: str, extra: list[str]):
    import socket
    import time
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    logp = os.path.join(cwd, "daemon.log")
    log = open(logp, "w")
    # line-buffered stdout so each request's lines can be told apart
    p = subprocess.Popen(["stdbuf", "-oL", os.path.join(HERE, "_ref", "bsgsd")] + BSGSD_ARGS + extra +
                         ["-t", "4", "-p", str(port), "-i", "127.0.0.1"], cwd=cwd, stdout=log, stderr=subprocess.STDOUT)
    t0 = time.time()
    while "Listening in" not in open(logp).read():
        assert p.poll() is None and time.time() - t0 < 300, "reference daemon did not start"
        time.sleep(0.2)
    return p, port, logp


def table_digests(d: str) -> dict:
    return {f: masked_table_digest(os.path.join(d, f)) for f in sorted(os.listdir(d)) if f != "daemon.log"}


def gen_bsgsd() -> None:
    import socket
    import time
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    out = {"args": BSGSD_ARGS, "requests": [], "starts": [],
           "_generator": "oracle/make_golden.py --bsgsd running oracle/_ref/bsgsd"}
    with tempfile.TemporaryDirectory() as td:
        p, port, logp = start_ref_daemon(td, [])
        for name, req in BSGSD_REQUESTS:
            before = len(open(logp).read())
            with socket.create_connection(("127.0.0.1", port), timeout=300) as c:
                c.sendall(req)
                reply = b""
                while True:
                    b = c.recv(4096)
                    if not b:
                        break
                    reply += b
            time.sleep(0.3)
            lines = [ln for ln in open(logp).read()[before:].split("\n")
                     if ln and not ln.startswith(("[+] Accepting", "[+] Closing"))]
            out["requests"].append({"name": name, "request": req.decode(), "reply": mask_elapsed(reply).decode(),
                                    "stdout": lines})
            print(name, reply[:60], lines, flush=True)
        p.kill()
        p.wait()
        out["keyfound"] = open(os.path.join(td, "KEYFOUNDKEYFOUND.txt")).read()
    d = None
    for name, extra, fresh in BSGSD_STARTS:
        if fresh:
            if d:
                shutil.rmtree(d)
            d = tempfile.mkdtemp()
        p, port, logp = start_ref_daemon(d, extra)
        p.kill()
        p.wait()
        msgs = [ln.strip() for ln in open(logp).read().split("\n") if "bP table" in ln]
        out["starts"].append({"name": name, "extra": extra, "fresh": fresh, "files": table_digests(d), "bptable_lines": msgs})
        print(name, out["starts"][-1], flush=True)
    shutil.rmtree(d)
    with open(os.path.join(REPO, "tests", "golden", "ref_bsgsd.json"), "w") as f:
        json.dump(out, f, indent=1)


# bsgsd's bloom-file options (bsgsd.cpp:776-889 parsing, 584-660 initBloomFilterMapped, 955-995
# --create-mapped, 1180-1255 the 3 x 256 shard filters bloom-%u.dat / bloom2-%u.dat / bloom3-%u.dat):
# sequences of daemon starts sharing one directory; each start serves one found request (when the
# daemon comes up) and is then stopped.  Recorded per start: whether it listened, its exit status
# when it did not, the [E]/[W] lines it printed, the reply, and every file it left (the -S files
# masked as in ref_bsgsd.json, the shard files per layer as in ref_mapped.json).
BSGSD_MAPPED_SEQS = [
    ("mapped_fresh_then_reload", [["--mapped"], ["--mapped"]]),
    ("mapped_then_load_bloom", [["--mapped"], ["--mapped", "--load-bloom"]]),
    ("load_bloom_missing", [["--mapped", "--load-bloom"]]),
    ("mapped_named_chunks", [["--mapped=named.dat", "--mapped-chunks", "4"], ["--mapped-chunks", "4"]]),
    ("mapped_size_override", [["--mapped-size", "64k"], ["--mapped-size", "64k"]]),
    ("bloom_bytes", [["--bloom-bytes", "100000"]]),
    ("create_then_mapped", [["--create-mapped=100000", "--bloom-file", "cm.dat"], ["--mapped", "--bloom-file", "cm.dat"]]),
    ("create_chunks", [["--create-mapped=100000", "--mapped-chunks", "4"]]),
    ("create_without_size", [["--create-mapped"]]),
    ("mapped_then_plain", [["--mapped"], []]),
    ("block_count_tmpdir_rmd_batch", [["--bsgs-block-count", "4", "--tmpdir", "tmpdir_x", "--rmd-batch-size", "8"],
                                      ["--bsgs-block-size", "1024"]]),
]


def bsgsd_dir_files(d: str) -> dict:
    """Every file in d: the 256 shard files of a layer (or of one chunk index of it) as one entry
    [sizes, sha256 of their concatenation], -S files by masked digest, others [size, sha256]."""
    import hashlib
    out, layers = {}, {}
    for f in sorted(os.listdir(d)):
        if not os.path.isfile(os.path.join(d, f)):
            continue
        m = re.match(r"(bloom[23]?-)(\d+)\.dat((?:\.\d+)?)$", f)
        if m:
            layers.setdefault(m.group(1) + "*.dat" + m.group(3), {})[int(m.group(2))] = f
        elif f.startswith("keyhunt_bsgs_"):
            out[f] = masked_table_digest(os.path.join(d, f))
        else:
            b = open(os.path.join(d, f), "rb").read()
            out[f] = [len(b), hashlib.sha256(b).hexdigest()]
    for key, shards in layers.items():
        h = hashlib.sha256()
        sizes = []
        for i in sorted(shards):
            b = open(os.path.join(d, shards[i]), "rb").read()
            sizes.append(len(b))
            h.update(b)
        out[key] = [sizes, h.hexdigest()]
        if len(shards) != 256:  # a start that stopped part-way through a layer
            out[key].append(sorted(shards))
    return out


def gen_bsgsd_mapped() -> None:
    import socket
    import time
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    res = {"args": BSGSD_ARGS, "request": BSGSD_REQUESTS[0][1].decode(),
           "_generator": "oracle/make_golden.py --bsgsd-mapped running oracle/_ref/bsgsd"}
    for name, starts in BSGSD_MAPPED_SEQS:
        steps = []
        with tempfile.TemporaryDirectory() as td:
            os.mkdir(os.path.join(td, "tmpdir_x"))
            for extra in starts:
                sk = socket.socket()
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
                sk.close()
                logp = os.path.join(td, "daemon.log")
                log = open(logp, "w")
                p = subprocess.Popen(["stdbuf", "-oL", os.path.join(HERE, "_ref", "bsgsd")] + BSGSD_ARGS + extra +
                                     ["-t", "4", "-p", str(port), "-i", "127.0.0.1"], cwd=td, stdout=log,
                                     stderr=subprocess.STDOUT)
                t0 = time.time()
                while "Listening in" not in open(logp).read() and p.poll() is None and time.time() - t0 < 300:
                    time.sleep(0.2)
                step = {"extra": extra, "listened": p.poll() is None}
                if step["listened"]:
                    with socket.create_connection(("127.0.0.1", port), timeout=300) as c:
                        c.sendall(BSGSD_REQUESTS[0][1])
                        reply = b""
                        while True:
                            b = c.recv(4096)
                            if not b:
                                break
                            reply += b
                    step["reply"] = reply.decode()
                    p.kill()
                p.wait()
                if not step["listened"]:
                    step["exit"] = p.returncode
                log.close()
                text = open(logp).read()
                step["notes"] = sorted(set(m.strip() for m in re.findall(r"\[[EW]\] [^\n]*", text)))
                os.remove(logp)
                for f in ("KEYFOUNDKEYFOUND.txt",):
                    if os.path.exists(os.path.join(td, f)):
                        os.remove(os.path.join(td, f))
                step["files"] = bsgsd_dir_files(td)
                step["tmpdir_files"] = sorted(os.listdir(os.path.join(td, "tmpdir_x")))
                steps.append(step)
                print(name, extra, step["listened"], step.get("exit"), repr(step.get("reply")), step["notes"],
                      {k: (v[0] if isinstance(v, list) and isinstance(v[0], int) else "...") for k, v in step["files"].items()},
                      step["tmpdir_files"], flush=True)
        res[name] = steps
    with open(os.path.join(REPO, "tests", "golden", "ref_bsgsd_mapped.json"), "w") as f:
        json.dump(res, f, indent=1)


# --mapped bloom files (keyhunt.cpp:724-806, 1131-1172, 1700-1785, 7630-7706; bloom/bloom.cpp:491-747):
# sequences of reference-CLI runs sharing one directory per sequence; after each run every mapped file
# is recorded (BSGS shard files per layer: their sizes and the sha256 of their concatenation).  The
# chunk count divides the 35,944-byte filter: with a remainder the reference maps the filter's last
# bytes to a chunk past the end (bloom.cpp:38-44) and crashes (-11).
RMD_ARGS = ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:100000", "-n", "0x100000", "-t", "4"]
BSGS_ARGS = ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "2", "-r", "7cce5efdac000000:7cce5efdad000000", "-t", "4"]
MAPPED_SEQS = [
    ("rmd160_fresh_then_reload", [RMD_ARGS + ["--mapped"], RMD_ARGS + ["--mapped"]]),
    ("rmd160_named_chunks", [RMD_ARGS + ["--mapped=tg.dat", "--mapped-chunks", "4"],
                             RMD_ARGS + ["--mapped=tg.dat", "--mapped-chunks", "4"]]),
    ("rmd160_size_override", [RMD_ARGS + ["--mapped-size", "1m"], RMD_ARGS + ["--mapped-size", "1m"]]),
    ("create_then_load", [["--create-mapped=100000", "--bloom-file", "cm.dat"],
                          RMD_ARGS + ["--mapped", "--bloom-file", "cm.dat", "--load-bloom"]]),
    ("xpoint_fresh", [["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:100000", "-n", "0x100000", "-t", "4", "--mapped"]]),
    ("vanity_fresh", [["-m", "vanity", "-v", "1Kha", "-v", "1PUB", "-l", "compress", "-r", "1:100000", "-n", "0x100000",
                       "-t", "4", "--mapped=v.dat"]]),
    ("eth_fresh", [["-m", "address", "-c", "eth", "-f", "eth_targets.txt", "-r", "1:100000", "-n", "0x100000", "-t", "4",
                    "--mapped"]]),
    ("bsgs_fresh_then_reload", [BSGS_ARGS + ["--mapped"], BSGS_ARGS + ["--mapped"]]),
    ("bsgs_size_override", [BSGS_ARGS + ["--mapped-size", "64k"]]),
    # -S with --mapped: a fresh run maps bloom.dat and writes data_<hex>.dat from that filter; a rerun reads
    # the data file and leaves bloom.dat alone; after a plain --mapped run the -S run reloads bloom.dat with
    # its size-derived geometry, which goes into the data file, and a plain -S run then reads that file
    ("rmd160_S_mapped_fresh_then_reload", [RMD_ARGS + ["-S", "--mapped"], RMD_ARGS + ["-S", "--mapped"]]),
    ("rmd160_mapped_then_S_mapped_then_S", [RMD_ARGS + ["--mapped"], RMD_ARGS + ["-S", "--mapped"], RMD_ARGS + ["-S"]]),
    # BSGS -S with --mapped: the reads are skipped (keyhunt.cpp:1983) but the table files are written from the
    # mapped shard filters (2504-2652), fresh and over reloaded shard files
    ("bsgs_S_mapped_fresh_then_rerun", [BSGS_ARGS + ["-S", "--mapped"], BSGS_ARGS + ["-S", "--mapped"]]),
    ("xpoint_S_mapped_override", [["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:100000", "-n", "0x100000", "-t", "4",
                                   "-S", "--mapped", "--mapped-size", "1m"]]),
    # -S with --mapped-chunks 4: the data file is hashed and written from the first chunk's mapping
    # (bloom.bf = bf_chunks[0], bloom.cpp:395) for bloom.bytes, past that mapping's end
    # (keyhunt.cpp:7770-7809): SIGBUS (-7) after the chunk files are filled and data_<hex>.dat is opened,
    # so the data file stays empty; the rerun fails reading it (7068, 1347) with exit 1
    ("rmd160_S_mapped_chunks", [RMD_ARGS + ["-S", "--mapped", "--mapped-chunks", "4"],
                                RMD_ARGS + ["-S", "--mapped", "--mapped-chunks", "4"]]),
]


def mapped_files(d: str) -> dict:
    import hashlib
    out, layers = {}, {}
    for f in sorted(os.listdir(d)):
        m = re.match(r"(bloom2?3?-)(\d+)\.dat$", f)
        if m:
            layers.setdefault(m.group(1), {})[int(m.group(2))] = f
        elif f.startswith("data_") and f.endswith(".dat"):  # -S target cache: its mmap pointer masked
            out[f] = [os.path.getsize(os.path.join(d, f)), masked_data_digest(os.path.join(d, f))]
        elif f.startswith("keyhunt_bsgs_"):  # -S table files: each shard's bf pointer masked
            out[f] = [os.path.getsize(os.path.join(d, f)), masked_table_digest(os.path.join(d, f))]
        elif f.endswith(".dat") or re.search(r"\.dat\.\d+$", f):
            b = open(os.path.join(d, f), "rb").read()
            out[f] = [len(b), hashlib.sha256(b).hexdigest()]
    for pfx, shards in layers.items():
        h = hashlib.sha256()
        sizes = []
        for i in range(256):
            b = open(os.path.join(d, shards[i]), "rb").read()
            sizes.append(len(b))
            h.update(b)
        out[pfx + "*"] = [sizes, h.hexdigest()]
    return out


def gen_mapped(only: list[str] | None = None) -> None:
    """--mapped [--only NAME ...]: with --only, just those sequences are rerun and merged into the file."""
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    out_path = os.path.join(REPO, "tests", "golden", "ref_mapped.json")
    res = json.load(open(out_path)) if only else {}
    res["_generator"] = "oracle/make_golden.py --mapped running oracle/_ref/keyhunt"
    for name, runs in MAPPED_SEQS:
        if only and name not in only:
            continue
        steps = []
        with tempfile.TemporaryDirectory() as td:
            for fn in os.listdir(DATA):
                shutil.copy(os.path.join(DATA, fn), td)
            for argv in runs:
                if os.path.exists(os.path.join(td, "KEYFOUNDKEYFOUND.txt")):
                    os.remove(os.path.join(td, "KEYFOUNDKEYFOUND.txt"))
                p = subprocess.run(["timeout", "300", REF_BIN] + argv + ["-q"], cwd=td, capture_output=True, text=True)
                text = ""
                for fn in ("KEYFOUNDKEYFOUND.txt", "VANITYKEYFOUND.txt"):
                    if os.path.exists(os.path.join(td, fn)):
                        text += open(os.path.join(td, fn)).read()
                        os.remove(os.path.join(td, fn))
                hits = sorted(parse_keyfound(text), key=lambda h: int(h["key"], 16))
                st = {"argv": argv, "exit": p.returncode, "hits": hits, "files": mapped_files(td)}
                if p.returncode:  # a failing run: the reference's [E] lines (stdout is lost on a signal)
                    st["stderr_E"] = [ln for ln in p.stderr.splitlines() if ln.startswith("[E]")]
                steps.append(st)
                print(name, argv[-3:], p.returncode, len(hits), {k: v[0] if k.endswith("*") is False else "..." for k, v in steps[-1]["files"].items()}, flush=True)
        res[name] = steps
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


# The reference's own stdout of single-thread runs (-t 1, so its print order is deterministic), for the
# output contract: the per-chunk "Base key" lines (keyhunt.cpp:3333-3346), the BSGS per-base
# "[+] Thread 0x..." lines (4618-4633, backward 6023-6035), with -M (FLAGMATRIX: one line each) and
# without -q (overwritten in place with \r), and the hit / "All points were found" / "End" text
# between them.  -s 0: no stats line.  tests/golden/data/bsgs_two_targets.txt = 63.pub + 125.txt (one
# target is never found, so the run walks every base and ends with "End").
STDOUT_RUNS = [
    ("rmd160_M", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:300000", "-n", "0x100000", "-M"]),
    ("rmd160_verbose", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:300000", "-n", "0x100000"]),
    ("rmd160_M_quiet", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:300000", "-n", "0x100000", "-M", "-q"]),
    ("rmd160_quiet", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:300000", "-n", "0x100000", "-q"]),
    ("address_M", ["-m", "address", "-f", "1to32.txt", "-r", "1:300000", "-n", "0x100000", "-M"]),
    ("xpoint_M", ["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:300000", "-n", "0x100000", "-M"]),
    ("xpoint_verbose", ["-m", "xpoint", "-f", "1to63_65.txt", "-r", "1:300000", "-n", "0x100000"]),
    ("bsgs_63_M", ["-m", "bsgs", "-f", "63.pub", "-r", "7cce5a0000000000:7cce9a0000000000", "-M"]),
    ("bsgs_63_verbose", ["-m", "bsgs", "-f", "63.pub", "-r", "7cce5a0000000000:7cce9a0000000000"]),
    ("bsgs_63_bases_M", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-r", "7cce5efdac000000:7cce5efdad000000", "-M"]),
    ("bsgs_63_bases_verbose", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-r", "7cce5efdac000000:7cce5efdad000000"]),
    ("bsgs_63_bases_quiet", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-r", "7cce5efdac000000:7cce5efdad000000", "-q"]),
    ("bsgs_63_backward_M", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-B", "backward", "-r", "7cce5efdac000000:7cce5efdad000000", "-M"]),
    ("bsgs_63_backward_verbose", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-B", "backward", "-r", "7cce5efdac000000:7cce5efdad000000"]),
    ("bsgs_two_M", ["-m", "bsgs", "-f", "bsgs_two_targets.txt", "-n", "0x100000", "-r", "7cce5efdac000000:7cce5efdad000000", "-M"]),
    ("bsgs_two_verbose", ["-m", "bsgs", "-f", "bsgs_two_targets.txt", "-n", "0x100000", "-r", "7cce5efdac000000:7cce5efdad000000"]),
]
# BSGS runs whose table-setup lines take other paths (keyhunt.cpp:1631-2700): -z above the 10000-item
# floor, and sequences run in ONE directory -- -S building then reading its files, --mapped creating
# then reloading its shard files, --ptable with --ptable-cache writing then --load-ptable reading
STDOUT_RUNS += [
    # the key is the last giant-step key of base 2 (base 2 + 2N), i.e. exactly base 3's start, which base 3
    # cannot reach (offset 0): the found line follows base 2's progress line
    ("bsgs_63_key_on_boundary_M", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-r", "7cce5efdac6f6808:7cce5efdad6f6808", "-M"]),
    ("bsgs_63_key_on_boundary_verbose", ["-m", "bsgs", "-f", "63.pub", "-n", "0x100000", "-r", "7cce5efdac6f6808:7cce5efdad6f6808"]),
    ("bsgs_63_z2_M", ["-m", "bsgs", "-f", "63.pub", "-k", "2", "-z", "2", "-r", "7cce5a0000000000:7cce9a0000000000", "-M"]),
]
_SMALL = ["-m", "bsgs", "-f", "63.pub", "-n", "0x1000000", "-k", "2", "-r", "7cce5efdac000000:7cce5efdad000000", "-M"]
STDOUT_SEQS = [
    ("bsgs_S_build_then_read", [_SMALL + ["-S"], _SMALL + ["-S"]]),
    ("bsgs_mapped_fresh_then_reload", [_SMALL + ["--mapped"], _SMALL + ["--mapped"]]),
    ("bsgs_ptable_cache_then_load", [_SMALL + ["--ptable", "c.tbl", "--ptable-cache"],
                                     _SMALL + ["--ptable", "c.tbl", "--ptable-cache", "--load-ptable"]]),
]
# the stats line (keyhunt.cpp:2904-2950) with and without -M: runs stopped after a few seconds; the
# fixture keeps the lines, the test compares their shape (numbers are the run's)
STATS_RUNS = [
    ("rmd160_stats_M", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:400000000", "-s", "1", "-M", "-q"], 4),
    ("rmd160_stats", ["-m", "rmd160", "-f", "1to32.rmd", "-l", "compress", "-r", "1:400000000", "-s", "1", "-q"], 4),
]
STATS_LINE = re.compile(rb"\r?\[\+\] Total \d+ keys in \d+ seconds: [^\r\n]*[\r\n]")


def gen_stdout(only: list[str] | None = None):
    """--stdout [--only NAME ...]: with --only, just those fixtures are rerun and merged into the file."""
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", "-j8"], check=True)
    out = os.path.join(REPO, "tests", "golden", "ref_stdout.json")
    res = json.load(open(out)) if only else {}
    res["_generator"] = "oracle/make_golden.py --stdout running oracle/_ref/keyhunt -t 1 -s 0"
    for name, argv in STDOUT_RUNS:
        if only and name not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            for fn in os.listdir(DATA):
                shutil.copy(os.path.join(DATA, fn), td)
            p = subprocess.run(["timeout", "300", REF_BIN] + argv + ["-t", "1", "-s", "0"], cwd=td, capture_output=True)
        res[name] = {"argv": argv, "exit": p.returncode, "stdout": p.stdout.decode("latin-1")}
        print(name, p.returncode, len(p.stdout), flush=True)
    for name, argvs in STDOUT_SEQS:
        if only and name not in only:
            continue
        runs = []
        with tempfile.TemporaryDirectory() as td:
            for fn in os.listdir(DATA):
                shutil.copy(os.path.join(DATA, fn), td)
            for argv in argvs:
                p = subprocess.run(["timeout", "300", REF_BIN] + argv + ["-t", "1", "-s", "0"], cwd=td, capture_output=True)
                runs.append({"argv": argv, "exit": p.returncode, "stdout": p.stdout.decode("latin-1")})
        res[name] = {"seq": runs}
        print(name, [(r["exit"], len(r["stdout"])) for r in runs], flush=True)
    for name, argv, secs in STATS_RUNS:
        if only and name not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            for fn in os.listdir(DATA):
                shutil.copy(os.path.join(DATA, fn), td)
            p = subprocess.run(["timeout", str(secs), REF_BIN] + argv + ["-t", "1"], cwd=td, capture_output=True)
        lines = [m.decode("latin-1") for m in STATS_LINE.findall(p.stdout)]
        res[name] = {"argv": argv, "stats_lines": lines}
        print(name, lines, flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--stdout", action="store_true")
    ap.add_argument("--vectors", action="store_true")
    ap.add_argument("--e2e", action="store_true")
    ap.add_argument("--tables", action="store_true")
    ap.add_argument("--data", action="store_true")
    ap.add_argument("--bsgsd", action="store_true")
    ap.add_argument("--mapped", action="store_true")
    ap.add_argument("--bsgsd-mapped", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    if not (a.vectors or a.e2e or a.tables or a.data or a.bsgsd or a.mapped or a.bsgsd_mapped or a.stdout):
        a.vectors = a.e2e = a.tables = a.data = a.bsgsd = a.mapped = a.bsgsd_mapped = a.stdout = True
    if a.vectors:
        gen_vectors()
    if a.e2e:
        gen_e2e(a.only)
    if a.tables:
        gen_tables()
    if a.data:
        gen_data()
    if a.bsgsd:
        gen_bsgsd()
    if a.mapped:
        gen_mapped(a.only)
    if a.bsgsd_mapped:
        gen_bsgsd_mapped()
    if a.stdout:
        gen_stdout(a.only)
