"""Deterministic target file with more than 10000 rows (the initBloomFilter floor,
keyhunt.cpp:7608), for -z (bloom size multiplier) parity: the 32 rows of 1to32.rmd followed by
12000 pseudo-random hash160s from a fixed seed.  Used by oracle/make_golden.py --data and by
tests/test_gpu_datafiles.py, which both write it with write(path)."""
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))


def write(path: str) -> None:
    rows = [l.strip() for l in open(os.path.join(HERE, "data", "1to32.rmd")) if l.strip()]
    rng = random.Random(0x6B657968)
    rows += ["%040x" % rng.getrandbits(160) for _ in range(12000)]
    with open(path, "w") as f:
        f.write("\n".join(rows) + "\n")


if __name__ == "__main__":
    import sys
    write(sys.argv[1])
