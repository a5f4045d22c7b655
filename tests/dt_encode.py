"""A small `.dt` writer for tests (no LZ4): turns an op list into the reference's wire format so
that synthetic documents can be round-tripped through the host decoder, the device decoder and
the device-staged checkout.

Format per SURVEY.md Appendix A / src/list/encoding/encode_oplog.rs (write_op :20-92, chunk
order :404-747), decode side decode_oplog.rs:590-960.  Ops are (agent, kind, pos, len, text,
parents) in LV order, as dt_amd.synth_ops returns them; every op is its own agent run and its
own graph entry (the decoder merges them back exactly like the builder API does).
"""
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


def encode_dt(agent_names, ops, del_content_unknown=False, ins_runs_per_op=False, unknown_every=0):
    """.dt bytes for `ops`.  del_content_unknown adds a delete PatchContent whose runs are all
    unknown; ins_runs_per_op writes one ContentIsKnown run per insert (else one run);
    unknown_every > 0 marks every n-th insert's content unknown (and leaves its text out)."""
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
    for agent, kind, pos, length, text, parents in ops:
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
            for k, p in enumerate(sorted(parents)):
                more = 1 if k + 1 < len(parents) else 0
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
