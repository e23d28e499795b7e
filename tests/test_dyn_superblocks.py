"""The dynamic super-block protocol of plk_jit_tree4 (csrc/plk_jit.hpp, the generated loop
head and the exit ticket), restated step by step and run under random interleavings of the
workgroups (CPU, no GPU): every super-block is computed exactly once, exactly one workgroup
finds itself last at the exit ticket, and it leaves the fragment's counter and the ticket
counter at 0 -- the state the next launch starts from (no host-side bookkeeping)."""
import random

import pytest

MASK = (1 << 32) - 1


def run_launch(n_sblocks, gx, ctr, rng, tickets=0):
    """One launch of gx workgroups over one fragment.  Workgroup state machine, as generated:
    pre-loop: thread 0 takes pend = atomic_add(ctr, 1); sb = blockIdx.x.
    loop while sb < n: (barrier) next = gx + pend if pend < n - gx else n;
                        (barrier) if next < n: pend = atomic_add(ctr, 1);
                        compute sb; sb = next.
    exit: t = atomic_add(tickets, 1); the workgroup with t == gx - 1 stores 0 to both counters."""
    done, lasts = [], []
    state = [{"sb": b, "pend": None, "phase": "grab0"} for b in range(gx)]
    live = list(range(gx))
    while live:
        w = rng.choice(live)
        s = state[w]
        if s["phase"] == "grab0":
            s["pend"], ctr = ctr, (ctr + 1) & MASK
            s["phase"] = "loop"
        elif s["phase"] == "loop":
            if s["sb"] >= n_sblocks:
                s["phase"] = "exit"
                continue
            d = s["pend"]
            nxt = gx + d if d < n_sblocks - gx else n_sblocks
            if nxt < n_sblocks:
                s["pend"], ctr = ctr, (ctr + 1) & MASK
            done.append(s["sb"])
            s["sb"] = nxt
        else:  # exit ticket
            t, tickets = tickets, tickets + 1
            if t == gx - 1:
                lasts.append(w)
                ctr, tickets = 0, 0
            live.remove(w)
    return done, ctr, tickets, lasts


@pytest.mark.parametrize("seed", range(12))
def test_every_superblock_once_and_counters_end_at_zero(seed):
    rng = random.Random(seed)
    ctr = tickets = 0
    for _ in range(5):  # consecutive launches, no host bookkeeping between them
        gx = rng.randint(1, 48)
        n = rng.randint(gx, 400)
        if n < 3 * gx:  # the host launches such a tier statically
            n = 3 * gx + rng.randint(0, 50)
        done, ctr, tickets, lasts = run_launch(n, gx, ctr, rng, tickets)
        assert sorted(done) == list(range(n))
        assert len(lasts) == 1
        assert ctr == 0 and tickets == 0


def test_stale_counter_never_leaves_the_range():
    """A counter that does not start at 0 (it cannot happen while every launch ends at its
    exit ticket; the kernel's range check is the guard) yields only in-range super-blocks or
    the end: no workgroup indexes past n_sblocks, none twice."""
    rng = random.Random(5)
    for off in (1, 7, 1000, MASK - 5):
        n, gx = 200, 20
        done, ctr, _, _ = run_launch(n, gx, off, rng)
        assert all(0 <= d < n for d in done)
        assert len(done) == len(set(done))
        assert ctr == 0  # and the launch's last workgroup repairs the counter
