"""Random linear histories (one agent, every op at the current version: one graph entry, the
reference's fast-forward case, merge.rs:811-840) for the fast-forward checkout tests.  Built with
the native ListOpLog (add_insert / add_delete_without_content, as crates/bench/src/utils.rs
builds the JSON traces) and encoded as .dt; the expected text is kept by a plain Python string
model alongside, and the tests also check it against the oracle."""
import random

import dt_amd

ALPHABET = "abcdefghij klmnop\nqrstuvwxyz" + "é" + "ß" + "€" + "中文" + "😀" + "🎉"


def random_linear(seed, n_ops, max_ins=12, paste_p=0.02, bs_p=0.15, unicode=True):
    """(encoded .dt bytes, expected text) of a random linear document with about n_ops edits:
    typing runs, pastes, forward deletes, backspace runs (merged into reversed delete runs) and
    the occasional delete of everything."""
    rng = random.Random(seed)
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("lin")
    text = []
    alpha = ALPHABET if unicode else "abcdefghij klmnopqrstuvwxyz\n"
    cursor = 0
    for _ in range(n_ops):
        r = rng.random()
        n = len(text)
        if n and r < bs_p:   # backspaces at the cursor: single-char deletes at decreasing positions
            k = rng.randint(1, min(8, n))
            cursor = min(max(cursor, 1), n)
            for _ in range(k):
                if cursor == 0:
                    break
                o.add_delete_without_content(a, cursor - 1, cursor)
                del text[cursor - 1]
                cursor -= 1
        elif n and r < bs_p + 0.12:   # forward delete of a range
            s = rng.randrange(n)
            e = min(n, s + rng.randint(1, 40))
            o.add_delete_without_content(a, s, e)
            del text[s:e]
            cursor = s
        elif n > 50 and r < bs_p + 0.125:   # select all, delete
            o.add_delete_without_content(a, 0, n)
            text = []
            cursor = 0
        else:
            if rng.random() < 0.3:
                cursor = rng.randint(0, n)
            cursor = min(cursor, n)
            k = rng.randint(200, 3000) if rng.random() < paste_p else rng.randint(1, max_ins)
            s = "".join(rng.choice(alpha) for _ in range(k))
            o.add_insert(a, cursor, s)
            text[cursor:cursor] = list(s)
            cursor += k
    return o.encode(), "".join(text).encode()


def sized_linear(n_runs, seed=0):
    """A linear document of exactly n_runs op runs (alternating inserts at the front and single
    deletes behind them, which never merge), for segment-boundary cases."""
    rng = random.Random(seed)
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("seg")
    text = []
    for k in range(n_runs):
        if k % 2 == 0 or not text:
            s = "".join(rng.choice("xyzw") for _ in range(rng.randint(1, 5)))
            p = rng.randint(0, len(text))
            o.add_insert(a, p, s)
            text[p:p] = list(s)
        else:
            p = rng.randrange(len(text))
            o.add_delete_without_content(a, p, p + 1)
            del text[p]
    return o.encode(), "".join(text).encode()
