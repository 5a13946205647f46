"""The device reduction's algorithm (kh_math.h fe_reduce512), restated in tests/_reduce_model.py:
its fast path is exact whenever no wave-level rare condition fires, its rare block is exact on
every input, and the generated operand pairs reach every V_j / W_i overflow."""
import random
from collections import Counter

from _reduce_model import P, fast, overflow_pairs, rare_block, reduce

EDGE = [P - 1 - k for k in range(24)] + [2**256 - 2**224 + k for k in range(24)] + \
       [2**k - 1 for k in range(224, 256)] + [2**255, 2**32, 1]


def _cases():
    rng = random.Random(11)
    cs = [rng.randrange(P) * rng.randrange(P) for _ in range(20000)]
    cs += [a * b for a, b in overflow_pairs()]
    cs += [a * b for a in EDGE for b in EDGE if a < P and b < P]
    return cs


def test_fast_path_exact_unless_rare():
    n_rare = 0
    for T in _cases():
        r, rare = fast(T)
        if rare:
            n_rare += 1
        else:
            assert r == T % P
    assert n_rare > 0


def test_rare_block_exact_everywhere():
    for T in _cases():
        assert rare_block(T) == T % P
        assert reduce(T) == T % P


def test_overflow_pairs_cover_every_slice():
    c = Counter(h for a, b in overflow_pairs() for h in fast(a * b)[1])
    for k in ("V0", "V2", "V4", "V6", "W1", "W3", "W5", "W7"):
        assert c[k] >= 8, (k, c)


def test_square_inputs_cover_slices():
    from _reduce_model import square_overflow_inputs
    xs = square_overflow_inputs()
    c = Counter(h for a in xs for h in fast(a * a)[1])
    for k in ("V2", "V4", "V6", "W1", "W3", "W5", "W7"):
        assert c[k] >= 2, (k, c)
    for a in xs:
        assert reduce(a * a) == a * a % P
