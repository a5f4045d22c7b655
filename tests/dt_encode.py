"""A small `.dt` writer for tests (no LZ4): turns an op list into the reference's wire format so
that synthetic documents can be round-tripped through the host decoder, the device decoder and
the device-staged checkout.

Format per SURVEY.md Appendix A / src/list/encoding/encode_oplog.rs (write_op :20-92, chunk
order :404-747), decode side decode_oplog.rs:590-960.  Ops are (agent, kind, pos, len, text,
parents) in LV order, as dt_amd.synth_ops returns them; every op is its own agent run and its
own graph entry (the decoder merges them back exactly like the builder API does).
"""
import random
import struct


def leb(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def zz_old(v):   # "old" sign-magnitude zigzag (leb.rs:286-323)
    return (abs(v) << 1) | (1 if v < 0 else 0)


def chunk(t, body):
    return leb(t) + leb(len(body)) + bytes(body)


def _crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_CRC = _crc_table()


def crc32c(data):   # CRC-32/ISCSI (src/encoding/tools.rs:111-115)
    c = 0xFFFFFFFF
    t = _CRC
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def write_op(kind, start, length, fwd, cursor):
    """encode_oplog.rs write_op: returns (bytes, new cursor)."""
    fwd = fwd or length == 1
    op_start = start + length if (kind == 1 and not fwd) else start
    op_end = start + length if (kind == 0 and fwd) else start
    diff = op_start - cursor
    if length != 1:
        n = length
        if kind == 1:
            n = (n << 1) | (1 if fwd else 0)
    elif diff != 0:
        n = zz_old(diff)
    else:
        n = 0
    n = (n << 1) | (1 if kind == 1 else 0)
    n = (n << 1) | (1 if diff != 0 else 0)
    n = (n << 1) | (1 if length != 1 else 0)
    out = leb(n)
    if length != 1 and diff != 0:
        out += leb(zz_old(diff))
    return out, op_end


def encode_dt(agent_names, ops, del_content_unknown=False, ins_runs_per_op=False, unknown_every=0,
              sort_parents=True, foreign_every=0):
    """.dt bytes for `ops`.  del_content_unknown adds a delete PatchContent whose runs are all
    unknown; ins_runs_per_op writes one ContentIsKnown run per insert (else one run);
    unknown_every > 0 marks every n-th insert's content unknown (and leaves its text out);
    sort_parents=False keeps each parent list in the given order (the decoder sorts it);
    foreign_every > 0 writes every n-th parent as a foreign (agent, seq) reference
    (decode_oplog.rs:880-890) instead of a local distance."""
    out = bytearray(b"DMNDTYPS") + leb(0)
    names = b"".join(leb(len(n.encode())) + n.encode() for n in agent_names)
    out += chunk(1, chunk(3, names))
    out += chunk(10, b"")
    seq = [0] * len(agent_names)
    versions, tp, hist = bytearray(), bytearray(), bytearray()
    ins_text, runs, del_runs = bytearray(), bytearray(), bytearray()
    ins_total = 0
    cursor = 0
    lv = 0
    n_ins = 0
    n_par = 0
    spans = []   # (lv, agent, seq) per op: a parent's (agent, seq) for foreign references
    for agent, kind, pos, length, text, parents in ops:
        spans.append((lv, agent, seq[agent]))
        versions += leb(((agent + 1) << 1) | 0) + leb(length)
        seq[agent] += length
        if kind == 0:
            b, cursor = write_op(0, pos, length, True, cursor)
            n_ins += 1
            unknown = unknown_every and n_ins % unknown_every == 0
            if not unknown:
                ins_text += text.encode()
            if ins_runs_per_op or unknown_every:
                runs += leb((length << 1) | (0 if unknown else 1))
            ins_total += length
        else:
            b, cursor = write_op(1, pos, length, True, cursor)
            del_runs += leb(length << 1)
        tp += b
        hist += leb(length)
        if not parents:
            hist += leb(1)   # foreign, n = 0: ROOT
        else:
            for k, p in enumerate(sorted(parents) if sort_parents else parents):
                more = 1 if k + 1 < len(parents) else 0
                n_par += 1
                if foreign_every and n_par % foreign_every == 0:
                    j = max(i for i, sp in enumerate(spans) if sp[0] <= p)
                    hist += leb(((spans[j][1] + 1) << 2) | (more << 1) | 1) + leb(spans[j][2] + p - spans[j][0])
                else:
                    hist += leb(((lv - p) << 2) | (more << 1))
        lv += length
    if not (ins_runs_per_op or unknown_every):
        runs = bytearray(leb((ins_total << 1) | 1)) if ins_total else bytearray()
    patches = bytearray()
    patches += chunk(24, leb(0) + chunk(13, leb(4) + bytes(ins_text)) + chunk(25, runs))
    if del_content_unknown:
        patches += chunk(24, leb(1) + chunk(13, leb(4)) + chunk(25, del_runs))
    patches += chunk(21, versions) + chunk(22, tp) + chunk(23, hist)
    out += chunk(20, patches)
    crc = crc32c(bytes(out))
    out += chunk(100, struct.pack("<I", crc))
    return bytes(out)


def graph_docs():
    """Documents whose histories stress the OpParents decode: merges of up to 12 parents in
    arbitrary order (duplicates included), foreign (agent, seq) parents, runs of single-parent
    spans (Graph::push extensions), ROOT parents, a frontier that grows past 64 (the device hands
    that document back: DECODE_DEFER) and one that grows to just under it."""
    out = []
    for doc in range(10):
        rng = random.Random(1000 + doc)
        na = 1 + doc % 5
        ops, lv, fr = [], 0, []
        wide = 70 if doc == 8 else (56 if doc == 9 else 0)
        for i in range(400):
            length = rng.choice([1, 1, 2, 5])
            if i < wide or not fr or rng.random() < 0.02:
                parents = []
            elif rng.random() < 0.35:
                parents = [lv - 1]
            elif rng.random() < 0.25:   # a fork from an interior version: a new frontier element
                parents = [rng.randrange(lv)]
            else:   # a merge of frontier elements, sometimes an interior version and a duplicate too
                parents = rng.sample(fr, min(rng.choice([1, 2, 2, 3, 4, 7, 12]), len(fr)))
                if rng.random() < 0.3:
                    parents.append(rng.randrange(lv))
                if rng.random() < 0.1:
                    parents.append(parents[0])
            ops.append((rng.randrange(na), 0, 0, length, "x" * length, parents))
            fr = [x for x in fr if x not in parents] + [lv + length - 1]
            lv += length
        out.append(encode_dt([f"g{i}" for i in range(na)], ops, sort_parents=(doc % 2 == 0),
                             foreign_every=(7 if doc % 3 == 1 else 0)))
    return out

