"""Model of k_hash_cand_1's pooled try-and-increment search (bls381_kernels.hpp,
BLS_HASH_COMPACT): the lane assignment and per-item resolution, simulated for a 64-lane wave
over random square patterns.  Each item must end with its lowest square offset -- the
spec's candidate order (bls_signature.md:74-86) -- whatever the other items do, and the
wave must finish in far fewer rounds than a lane-per-item loop's slowest item.
"""
import random


def nth_set_bit(m, r):
    for b in range(64):
        if (m >> b) & 1:
            if r == 0:
                return b
            r -= 1
    raise AssertionError("rank out of range")


def pooled_search(is_square, valid):
    """is_square(item, offset) -> bool; valid[lane]; returns (found offsets, rounds)"""
    k = [0] * 64
    found = [-1 if valid[i] else 0 for i in range(64)]
    rounds = 0
    while True:
        P = sum(1 << i for i in range(64) if found[i] < 0)
        if P == 0:
            return found, rounds
        rounds += 1
        m = bin(P).count("1")
        t = [nth_set_bit(P, lane % m) for lane in range(64)]
        off = [k[t[lane]] + lane // m for lane in range(64)]
        B = sum(1 << lane for lane in range(64) if is_square(t[lane], off[lane]))
        for lane in range(64):
            if found[lane] < 0:
                r = bin(P & ((1 << lane) - 1)).count("1")
                first, cnt, j = -1, 0, r
                while j < 64:
                    if first < 0 and (B >> j) & 1:
                        first = cnt
                    j += m
                    cnt += 1
                if first >= 0:
                    found[lane] = k[lane] + first
                else:
                    k[lane] += cnt


def test_pooled_search_finds_first_square():
    rng = random.Random(0x5EA2C4)
    total_rounds = 0
    for trial in range(300):
        squares = [[rng.random() < 0.5 for _ in range(200)] for _ in range(64)]
        if trial % 7 == 0:                       # some items with long runs of non-squares
            for i in rng.sample(range(64), 5):
                run = rng.randrange(10, 60)
                squares[i][:run] = [False] * run
        valid = [True] * 64 if trial % 5 else [i < rng.randrange(1, 64) for i in range(64)]
        found, rounds = pooled_search(lambda i, o: squares[i][o], valid)
        total_rounds += rounds
        for i in range(64):
            if valid[i]:
                assert found[i] == squares[i].index(True), (trial, i)
    # a lane-per-item loop needs ~7.3 rounds per wave at probability 1/2; the pool needs ~3
    assert total_rounds / 300 < 4.5
