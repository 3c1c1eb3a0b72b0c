"""The entropy coder's word hand-over between workgroups (p64vlc.hip,
k_vlc_blk, VLC_ONE / VLC_GIVEN), restated in Python and checked on random
and degenerate ranges: empty workgroups (an invalid record leaves a range
without a bit), ranges inside one word, several workgroups sharing a word,
ranges starting or ending on word boundaries.  Every picture word must be
written exactly once and hold the OR of every workgroup's bits in it.

This restates the kernel's rules (the `sh_first` / `sh_last` / one-word
branches at the end of k_vlc_blk); the GPU tests check the kernel's output
itself (tests/test_gpu_stream.py)."""
import random

import pytest


def wg_bits(first, n, seed):
    """a workgroup's bits: n random bits from picture bit `first`, as {word: value}"""
    rng = random.Random(seed)
    words = {}
    for i in range(n):
        if rng.random() < 0.5:
            p = first + i
            words[p >> 5] = words.get(p >> 5, 0) | (1 << (31 - (p & 31)))
    return words


def run_protocol(phase, totals, order_seed):
    ng = len(totals)
    firsts = []
    f = phase
    for t in totals:
        firsts.append(f)
        f += t
    bits = [wg_bits(firsts[g], totals[g], 1000 + g) for g in range(ng)]
    out, writes, tails = {}, {}, {}

    def store(w, v):
        writes[w] = writes.get(w, 0) + 1
        out[w] = v

    # workgroups finish in any order, but one that needs the previous tail
    # waits for it (the kernel spins): process in a random order, deferring
    # until the tail it needs exists
    pending = list(range(ng))
    random.Random(order_seed).shuffle(pending)
    progress = True
    while pending and progress:
        progress = False
        for g in list(pending):
            first, wt = firsts[g], totals[g]
            endb = first + wt
            w0, wl = first >> 5, (endb - 1) >> 5
            sh_first = g > 0 and (first & 31) != 0
            sh_last = g < ng - 1 and (endb & 31) != 0
            if sh_first and (g - 1) not in tails:
                continue  # (spins until the previous workgroup publishes its tail)
            mine = bits[g]
            if wt > 0 and w0 != wl:
                for w in range(w0, wl + 1):
                    if not (w == w0 and sh_first) and not (w == wl and sh_last):
                        store(w, mine.get(w, 0))
                if sh_last:
                    tails[g] = mine.get(wl, 0)
                if sh_first:
                    store(w0, mine.get(w0, 0) | tails[g - 1])
            else:  # one word (or none): the previous tail and ours
                v = mine.get(w0, 0) if wt > 0 else 0
                if sh_first:
                    v |= tails[g - 1]
                if sh_last:
                    tails[g] = v
                elif wt > 0 or sh_first:
                    store(w0, v)
            pending.remove(g)
            progress = True
    assert not pending, "a workgroup waits for a tail nobody publishes"
    want = {}
    for m in bits:
        for w, v in m.items():
            want[w] = want.get(w, 0) | v
    end = phase + sum(totals)
    used = set(range(phase >> 5, ((end - 1) >> 5) + 1)) if end > phase else set()
    if phase & 31 and end > phase:
        pass  # (word 0's leading phase bits are zeros the first workgroup writes)
    assert set(writes) == used, "every word of the picture written"
    assert all(c == 1 for c in writes.values()), "no word written twice"
    for w in used:
        assert out[w] == want.get(w, 0), f"word {w}"


@pytest.mark.parametrize("case", range(200))
def test_vlc_word_handover_random(case):
    rng = random.Random(case)
    ng = rng.randint(1, 12)
    kinds = [lambda: rng.randint(0, 3), lambda: rng.randint(1, 40), lambda: rng.randint(30, 400),
             lambda: 32 * rng.randint(1, 5), lambda: 0]
    totals = [rng.choice(kinds)() for _ in range(ng)]
    totals[0] = max(totals[0], 1)  # (the picture header: the first workgroup always has bits)
    run_protocol(rng.randint(0, 7), totals, case)


@pytest.mark.parametrize("totals,phase", [
    ([41, 0, 0, 5], 3),        # empty workgroups between: the tail passes through them
    ([32, 32, 32], 0),         # every range ends on a word boundary: nothing shared
    ([10, 3, 2, 1, 40], 7),    # several workgroups inside one word
    ([33, 31, 1], 0),          # a range ending exactly on a boundary after a shared start
    ([5], 2),                  # one workgroup, one word
])
def test_vlc_word_handover_edges(totals, phase):
    for order in range(6):
        run_protocol(phase, totals, order)
