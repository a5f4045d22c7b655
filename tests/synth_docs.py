"""Synthetic oplogs for the cut-replay tests (test data generators, not the oracle)."""
import random

import dt_amd


def phased_doc(seed, phases=14):
    """Concurrent phases joined by linear stretches: each phase forks 2-3 branches off one
    version (branch 0 inserts and deletes, the others only insert, so the merged length is
    known), then a linear stretch continues from the merge -- cut points between phases,
    concurrency right up to them."""
    rng = random.Random(seed)
    o = dt_amd.ListOpLog()
    agents = [o.get_or_create_agent_id(n) for n in ("ann", "bob", "cyd")]
    length = 0
    alpha = "abcdefghijklmnopqrstuvwxyz"
    for _ in range(phases):
        fork = list(o.local_frontier())
        added = 0
        for j in range(rng.choice((2, 3))):
            par, blen = fork, length
            for _ in range(rng.randint(3, 9)):
                if j == 0 and blen > 4 and rng.random() < 0.35:
                    a = rng.randrange(blen - 1)
                    b = min(blen, a + rng.randint(1, 4))
                    lv = o.add_delete_at(agents[j], par, a, b)
                    blen -= b - a
                    added -= b - a
                else:
                    t = "".join(rng.choice(alpha) for _ in range(rng.randint(1, 6)))
                    lv = o.add_insert_at(agents[j], par, rng.randint(0, blen), t)
                    blen += len(t)
                    added += len(t)
                par = [lv]
        length += added
        for _ in range(rng.randint(2, 8)):   # linear stretch from the merge
            a = rng.choice(agents)
            if length > 4 and rng.random() < 0.3:
                s0 = rng.randrange(length - 1)
                e0 = min(length, s0 + rng.randint(1, 3))
                o.add_delete_without_content(a, s0, e0)
                length -= e0 - s0
            else:
                t = "".join(rng.choice(alpha) for _ in range(rng.randint(1, 8)))
                o.add_insert(a, rng.randint(0, length), t)
                length += len(t)
    return o.encode()
