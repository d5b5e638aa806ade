"""The closing commit's append protocol on one counter (csrc/gc_internal.h gc_stage_flush,
csrc/gc_kernels.hip gc_stage_flush_ticket), modelled with random interleavings of the
workgroups' atomics: waves flush full LDS stages mid-launch (count), every workgroup ends with
one arrival ticket (count + 2^40), the last arrival closes.  With the count masked out of the
returned value (GC_COUNT_MASK) every entry lands in [0, total) exactly once and the last
workgroup sees the total; without the mask a flush that follows an early ticket writes
k * 2^40 entries past the list -- round 3's fault on the 10M uniform graph."""
import random

import pytest

SHIFT = 40
MASK = (1 << SHIFT) - 1
CAP = 512  # GC_STAGE_CAP


def run(pushes, seed, masked):
    """pushes[w][i]: entries wave i of workgroup w pushes; returns (written slots, total seen by
    the last arrival, number of last arrivals)."""
    rng = random.Random(seed)
    cnt = 0
    written = []
    # each workgroup: a program of atomics -- its waves' mid-launch flushes (full stages), then
    # the ticket carrying every wave's remainder
    progs = []
    for w, waves in enumerate(pushes):
        ops = []
        rest = 0
        for p in waves:
            full, r = divmod(p, CAP)
            ops += [("flush", CAP)] * full
            rest += r
        rng.shuffle(ops)  # the waves' flushes interleave
        ops.append(("ticket", rest))
        progs.append(ops)
    lasts, total_seen = 0, None
    live = [w for w in range(len(progs))]
    while live:
        w = rng.choice(live)
        kind, c = progs[w].pop(0)
        old = cnt
        if kind == "flush":
            cnt += c
            base = old & MASK if masked else old
            written += range(base, base + c)
        else:
            cnt += (1 << SHIFT) | c
            base = old & MASK
            written += range(base, base + c)
            if (old >> SHIFT) == len(progs) - 1:
                lasts += 1
                total_seen = base + c
        if not progs[w]:
            live.remove(w)
    return written, total_seen, lasts


@pytest.mark.parametrize("seed", range(20))
def test_masked_flushes_fill_the_list_exactly(seed):
    rng = random.Random(1000 + seed)
    G = rng.randint(2, 40)
    pushes = [[rng.choice([0, 3, 100, 511, 512, 640, 1500]) for _ in range(4)] for _ in range(G)]
    written, total, lasts = run(pushes, seed, masked=True)
    n = sum(sum(w) for w in pushes)
    assert lasts == 1 and total == n
    assert sorted(written) == list(range(n))


def test_unmasked_flush_after_a_ticket_writes_past_the_list():
    # an idle workgroup (only its ticket) and busy ones whose waves overflow their stages (640
    # pushes: one mid-launch flush each); some interleaving puts a flush after the idle ticket
    pushes = [[0, 0, 0, 0]] + [[640, 640, 0, 0]] * 3
    for seed in range(50):
        written, _, _ = run(pushes, seed, masked=False)
        if max(written) >= 1 << SHIFT:
            return
    pytest.fail("no interleaving put a flush after a ticket")
