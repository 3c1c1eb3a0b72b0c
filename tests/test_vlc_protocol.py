"""The entropy coder's word hand-over between workgroups (p64vlc.hip,
k_vlc_blk, VLC_ONE / VLC_GIVEN), restated in Python and checked on random
and degenerate ranges: empty workgroups (an invalid record leaves a range
without a bit), ranges inside one word, several workgroups sharing a word,
ranges starting or ending on word boundaries.  Every picture word must be
written exactly once and hold the OR of every workgroup's bits in it.

Two levels of the model:
* run_protocol: the LDS path's rules (the `sh_first` / `sh_last` / one-word
  branches at the end of k_vlc_blk), workgroups completing in any order.
* run_interleaved: every workgroup as a sequence of memory operations (zero
  store, atomic OR, read, store, tail publish / wait) run by an adversarial
  scheduler that interleaves single operations of all workgroups at random
  -- including the big path (a wave past its 8,160-bit LDS copy zeroes its
  words and ORs its codes straight into memory).  The kernel's big path
  keeps the shared first/last words in LDS (BitWriter s0/s1, round 6);
  `racy=True` restates the round-5 big path, which zeroed and ORed the
  shared words in memory, and the model must catch that race.

This restates the kernel's rules; the GPU tests check the kernel's output
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


def layout(phase, totals):
    firsts = []
    f = phase
    for t in totals:
        firsts.append(f)
        f += t
    return firsts


def expected(bits, phase, totals):
    want = {}
    for m in bits:
        for w, v in m.items():
            want[w] = want.get(w, 0) | v
    end = phase + sum(totals)
    used = set(range(phase >> 5, ((end - 1) >> 5) + 1)) if end > phase else set()
    return want, used


def run_protocol(phase, totals, order_seed):
    ng = len(totals)
    firsts = layout(phase, totals)
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
    want, used = expected(bits, phase, totals)
    assert set(writes) == used, "every word of the picture written"
    assert all(c == 1 for c in writes.values()), "no word written twice"
    for w in used:
        assert out[w] == want.get(w, 0), f"word {w}"


# ---------------------------------------------------------------------------
# operation-level model with an adversarial scheduler

class Mem:
    def __init__(self):
        self.words = {}      # picture word -> value (None = never written)
        self.owner = {}      # picture word -> set of workgroups that wrote it
        self.incl = set()    # workgroups that published their end (look-back)
        self.tails = {}      # workgroup -> published tail


def workgroup_ops(g, ng, first, wt, mine, big, racy):
    """k_vlc_blk's memory operations of workgroup g after its look-back, one
    yield per operation.  A yielded ("wait_incl", g-1) or ("wait_tail", g-1)
    blocks until that workgroup has published."""
    endb = first + wt
    w0, wl = first >> 5, (endb - 1) >> 5
    sh_first = g > 0 and (first & 31) != 0
    sh_last = g < ng - 1 and (endb & 31) != 0
    if g > 0:
        yield ("wait_incl", g - 1)   # the look-back: the previous end is known
    yield ("publish_incl", g)        # line `st_store(stw + 2*G, ST_INCL ...)`
    firstv = lastv = 0
    if wt > 0 and not big:           # the LDS path: unshared words stored once
        for w in range(w0, wl + 1):
            if not (w == w0 and sh_first) and not (w == wl and sh_last):
                yield ("store", w, mine.get(w, 0))
        firstv, lastv = mine.get(w0, 0), mine.get(wl, 0)
    elif wt > 0:                     # the big path
        assert w0 != wl
        lds = {}
        for w in range(w0, wl + 1):
            shared = (w == w0 and sh_first) or (w == wl and sh_last)
            if racy or not shared:
                yield ("store", w, 0)    # zeroing
        for w in range(w0, wl + 1):      # the codes, word by word (atomic ORs)
            v = mine.get(w, 0)
            shared = (w == w0 and sh_first) or (w == wl and sh_last)
            if not racy and shared:
                lds[w] = lds.get(w, 0) | v
            elif v:
                yield ("or", w, v)
        if racy:
            firstv = yield ("read", w0)
            lastv = yield ("read", wl)
        else:
            firstv, lastv = lds.get(w0, 0), lds.get(wl, 0)
    if wt == 0 or w0 == wl:
        v = firstv if wt > 0 else 0
        if sh_first:
            v |= (yield ("wait_tail", g - 1))
        if sh_last:
            yield ("publish_tail", g, v)
        elif wt > 0 or sh_first:
            yield ("store", w0, v)
    else:
        if sh_last:
            yield ("publish_tail", g, lastv)
        if sh_first:
            pv = yield ("wait_tail", g - 1)
            yield ("store", w0, firstv | pv)


def run_interleaved(phase, totals, bigs, sched_seed, racy=False):
    """Returns (ok, message): the picture words after an adversarial
    interleaving of every workgroup's operations."""
    ng = len(totals)
    firsts = layout(phase, totals)
    bits = [wg_bits(firsts[g], totals[g], 1000 + g) for g in range(ng)]
    mem = Mem()
    gens = [workgroup_ops(g, ng, firsts[g], totals[g], bits[g], bigs[g], racy) for g in range(ng)]
    pending_op = [None] * ng
    reply = [None] * ng
    for g in range(ng):
        pending_op[g] = next(gens[g], None)
    rng = random.Random(sched_seed)
    while any(op is not None for op in pending_op):
        ready = []
        for g, op in enumerate(pending_op):
            if op is None:
                continue
            if op[0] == "wait_incl" and op[1] not in mem.incl:
                continue
            if op[0] == "wait_tail" and op[1] not in mem.tails:
                continue
            ready.append(g)
        if not ready:
            return False, "deadlock"
        g = rng.choice(ready)
        op = pending_op[g]
        res = None
        if op[0] == "publish_incl":
            mem.incl.add(op[1])
        elif op[0] == "store":
            mem.words[op[1]] = op[2]
            mem.owner.setdefault(op[1], set()).add(g)
        elif op[0] == "or":
            mem.words[op[1]] = (mem.words.get(op[1]) or 0) | op[2]
            mem.owner.setdefault(op[1], set()).add(g)
        elif op[0] == "read":
            res = mem.words.get(op[1]) or 0
        elif op[0] == "publish_tail":
            mem.tails[op[1]] = op[2]
        elif op[0] == "wait_tail":
            res = mem.tails[op[1]]
        try:
            pending_op[g] = gens[g].send(res)
        except StopIteration:
            pending_op[g] = None
    want, used = expected(bits, phase, totals)
    if set(mem.words) != used:
        return False, "words written != the picture's words"
    for w in used:
        if mem.words[w] != want.get(w, 0):
            return False, f"word {w}: {mem.words[w]:#x} != {want.get(w, 0):#x}"
    if not racy and any(len(o) != 1 for o in mem.owner.values()):
        return False, "a word touched by two workgroups"
    return True, ""


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


def _big_case(case):
    """ranges of which some are 'big' (the kernel's big path: > 8,160 bits in
    a wave; the model only needs a multi-word range, so sizes stay small)"""
    rng = random.Random(7000 + case)
    ng = rng.randint(2, 8)
    totals, bigs = [], []
    for _ in range(ng):
        big = rng.random() < 0.6
        totals.append(rng.randint(40, 300) if big else rng.choice([0, rng.randint(1, 40), rng.randint(30, 200)]))
        bigs.append(big)
    totals[0] = max(totals[0], 40)
    return rng.randint(0, 7), totals, bigs


@pytest.mark.parametrize("case", range(60))
def test_vlc_big_path_interleaved(case):
    """the round-6 big path under 25 adversarial schedules each: every word
    exact, touched in memory by one workgroup only"""
    phase, totals, bigs = _big_case(case)
    for s in range(25):
        ok, msg = run_interleaved(phase, totals, bigs, 100 * case + s)
        assert ok, (msg, phase, totals, bigs, s)


def test_vlc_lds_path_interleaved():
    for case in range(40):
        phase, totals, _ = _big_case(case)
        for s in range(10):
            ok, msg = run_interleaved(phase, totals, [False] * len(totals), s)
            assert ok, (msg, phase, totals, s)


def test_model_catches_round5_big_path_race():
    """the round-5 big path (shared words zeroed and ORed in memory) loses
    bits under some interleaving: the model must find one"""
    found = False
    for case in range(60):
        phase, totals, bigs = _big_case(case)
        for s in range(25):
            ok, _ = run_interleaved(phase, totals, bigs, 100 * case + s, racy=True)
            if not ok:
                found = True
                break
        if found:
            break
    assert found
