"""Sequential Python model of dt_ff.hip (the linear-history checkout): the same segments of
FF_RUNS op runs, the same piece lists (src, len, pos) with placeholder pieces, the same pairwise
composition per level and the same byte-offset pass.  Test infrastructure: it checks the
algorithm on the CPU against the oracle's fast-forward checkout (merge.rs:811-840) without a
GPU; the kernel is checked against the same oracle on the GPU (tests/test_gpu_ff.py).
"""
FF_RUNS = 63
FF_PIECES = 128
PH = 0x80000000


class ModelError(Exception):
    pass


def segment(runs, lin):
    """One segment's replay: runs = [(lv, len, pos, kind)], kind 0 insert / 1 delete, applied to
    a text of lin placeholder chars.  Returns the piece list [(src, len, pos)]."""
    pieces = [(PH, lin)] if lin else []
    for lv, ln, pos, kind in runs:
        total = sum(p[1] for p in pieces)
        if kind == 0:
            if pos > total:
                raise ModelError("insert past the end")
            e, k, off = 0, len(pieces), 0
            for j, (s, l) in enumerate(pieces):
                if e <= pos < e + l:
                    k, off = j, pos - e
                    break
                e += l
            if off == 0 and k > 0 and not pieces[k - 1][0] & PH and sum(pieces[k - 1]) == lv:
                s, l = pieces[k - 1]
                pieces[k - 1] = (s, l + ln)
                continue
            if off == 0:
                pieces[k:k] = [(lv, ln)]
            else:
                s, l = pieces[k]
                pieces[k:k + 1] = [(s, off), (lv, ln), (s + off, l - off)]
        else:
            de = pos + ln
            if de > total:
                raise ModelError("delete past the end")
            out, e = [], 0
            for s, l in pieces:
                a, b = e, e + l
                if a < pos:
                    out.append((s, min(b, pos) - a))
                if b > de:
                    out.append((s + (max(a, de) - a), b - max(a, de)))
                e = b
            pieces = out
        if len(pieces) > FF_PIECES:
            raise ModelError("piece slots exceeded")
    res, e = [], 0
    for s, l in pieces:
        res.append((s, l, e))
        e += l
    return res


def compose(A, B):
    """B applied on top of A's text: B's placeholder pieces expanded into A's pieces."""
    out = []
    for s, l, p in B:
        if not s & PH:
            out.append((s, l, p))
            continue
        x, y = s & ~PH, (s & ~PH) + l
        for a_s, a_l, a_p in A:
            x0, x1 = max(a_p, x), min(a_p + a_l, y)
            if x0 < x1:
                out.append((a_s + (x0 - a_p), x1 - x0, p + (x0 - x)))
    return out


def checkout(ops, cbyte, content):
    """ops: decoder quads (lv, len, pos, kind | fwd << 1); cbyte: per-LV byte offsets; content:
    inserted UTF-8.  The text bytes, built as the kernels build them."""
    runs = [(o[0], o[1], o[2], o[3] & 1) for o in ops]
    segs = [runs[k:k + FF_RUNS] for k in range(0, len(runs), FF_RUNS)]
    lists, lin = [], 0
    for sg in segs:
        lists.append(segment(sg, lin))
        lin += sum(r[1] if r[3] == 0 else -r[1] for r in sg)
    while len(lists) > 1:   # one level: pairs (2i, 2i+1), a lone last group carried over
        nxt = []
        for k in range(0, len(lists), 2):
            if k + 1 < len(lists):
                c = compose(lists[k], lists[k + 1])
                if len(c) > len(lists[k]) + len(lists[k + 1]):
                    raise ModelError("composition outgrew its slots")
                nxt.append(c)
            else:
                nxt.append(lists[k])
        lists = nxt
    out = bytearray()
    for s, l, _ in (lists[0] if lists else []):
        if s & PH:
            raise ModelError("placeholder in the final list")
        c0, cl = cbyte[s], cbyte[s + l - 1]
        n = 1 if content[cl] < 0x80 else 2 if content[cl] & 0xE0 == 0xC0 else 3 if content[cl] & 0xF0 == 0xE0 else 4
        out += content[c0:cl + n]
    return bytes(out)
