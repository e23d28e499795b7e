"""The dynamic super-block protocol of plk_jit_tree4 (csrc/plk_jit.hpp, the generated loop
head; csrc/plk.hip, the host's counter base), restated step by step and run under random
interleavings of the workgroups (CPU, no GPU): every super-block is computed exactly once,
and each fragment's counter ends the launch at base + n_sblocks -- the value the host adds
for the next launch -- including across the 32-bit wrap of the counter."""
import random

import pytest

MASK = (1 << 32) - 1


def run_launch(n_sblocks, gx, base, ctr, rng):
    """One launch of gx workgroups over one fragment.  Workgroup state machine, as generated:
    pre-loop: thread 0 takes pend = atomic_add(ctr, 1); sb = blockIdx.x.
    loop while sb < n: (barrier) next = gx + (pend - base) if that difference < n - gx else n;
                        (barrier) if next < n: pend = atomic_add(ctr, 1);
                        compute sb; sb = next."""
    done = []
    state = []
    for b in range(gx):
        state.append({"sb": b, "pend": None, "phase": "grab0"})
    live = list(range(gx))
    while live:
        w = rng.choice(live)
        s = state[w]
        if s["phase"] == "grab0":
            s["pend"], ctr = ctr, (ctr + 1) & MASK
            s["phase"] = "loop"
        elif s["phase"] == "loop":
            if s["sb"] >= n_sblocks:
                live.remove(w)
                continue
            d = (s["pend"] - base) & MASK
            nxt = gx + d if d < n_sblocks - gx else n_sblocks
            if nxt < n_sblocks:
                s["pend"], ctr = ctr, (ctr + 1) & MASK
            done.append(s["sb"])
            s["sb"] = nxt
    return done, ctr


@pytest.mark.parametrize("seed", range(12))
def test_every_superblock_once_and_counter_ends_at_base_plus_n(seed):
    rng = random.Random(seed)
    base = rng.choice([0, 12345, MASK - 40, MASK - 3])  # (also across the 32-bit wrap)
    ctr = base
    for _ in range(5):  # consecutive launches, the host adding n_sblocks each time
        gx = rng.randint(1, 48)
        n = rng.randint(gx, 400)
        if n < 3 * gx:  # the host launches such a tier statically
            n = 3 * gx + rng.randint(0, 50)
        done, ctr = run_launch(n, gx, base, ctr, rng)
        assert sorted(done) == list(range(n))
        base = (base + n) & MASK
        assert ctr == base


def test_stale_counter_never_leaves_the_range():
    """A counter that does not hold the expected base (it cannot happen while the host's
    bookkeeping holds; the kernel's range check is the guard) yields only in-range
    super-blocks or the end: no workgroup indexes past n_sblocks."""
    rng = random.Random(5)
    for off in (1, 7, 1000, MASK - 5):
        n, gx, base = 200, 20, 777
        done, _ = run_launch(n, gx, base, (base + off) & MASK, rng)
        assert all(0 <= d < n for d in done)
        assert len(done) == len(set(done))
