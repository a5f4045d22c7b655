"""Sequential Python model of dt_replay.hip (same blocked data structure, same command
semantics, lanes as loops).  Test/debug infrastructure: it lets the kernel's algorithm be
checked on the CPU against the oracle, command by command, without a GPU.
"""
BLK = 64
SB = 64
ROOT_ID = 0xFFFFFFFF
END_ID = 0xFFFFFFFE
DEL_BIT = 0x80
MASK64 = (1 << 64) - 1


class ModelError(Exception):
    pass


def popc(x):
    return bin(x).count("1")


class Doc:
    def __init__(self, cmds, n_lv, cbyte, content, aruns, max_blocks):
        self.cmds, self.n_lv, self.cbyte, self.content, self.aruns = cmds, n_lv, cbyte, content, aruns
        self.max_blocks = max_blocks
        self.st = [0] * n_lv
        self.blk = [0] * n_lv
        self.slot = [0] * n_lv
        self.aux = [0] * n_lv
        self.orr = [0] * n_lv
        self.items = [[0] * BLK for _ in range(max_blocks)]
        self.mvis = [0] * max_blocks
        self.mlive = [0] * max_blocks
        self.bcnt = [0] * max_blocks
        self.ord = [0] * max_blocks
        self.opos = [0] * max_blocks
        nsb = (max_blocks + SB - 1) // SB
        self.svis = [0] * nsb
        self.scnt = [0] * nsb
        self.nb = 1

    def nsb(self):
        return (self.nb + SB - 1) // SB

    # ---- queries
    def find_vis(self, p):
        base = 0
        for sb in range(self.nsb()):
            if base + self.svis[sb] > p:
                break
            base += self.svis[sb]
        else:
            raise ModelError(f"find_vis({p}) past end")
        for i in range(sb * SB, min(self.nb, sb * SB + SB)):
            b = self.ord[i]
            v = popc(self.mvis[b])
            if base + v > p:
                off = p - base
                mv = self.mvis[b]
                for s in range(BLK):
                    if (mv >> s) & 1:
                        if off == 0:
                            return b, s
                        off -= 1
                raise ModelError("select failed")
            base += v
        raise ModelError(f"find_vis({p}) superblock mismatch")

    def rank_of(self, item):
        b, s = self.blk[item], self.slot[item]
        p = self.opos[b]
        sb = p // SB
        acc = sum(self.scnt[:sb])
        acc += sum(self.bcnt[self.ord[i]] for i in range(sb * SB, p))
        return acc + s

    def normalize(self, b, s):
        while s >= self.bcnt[b]:
            p = self.opos[b] + 1
            if p >= self.nb:
                return b, s
            b, s = self.ord[p], 0
        return b, s

    def next_live(self, b, s):
        ml = self.mlive[b] & (MASK64 << s) & MASK64 if s < 64 else 0
        if ml:
            return b, (ml & -ml).bit_length() - 1
        for p in range(self.opos[b] + 1, self.nb):
            bb = self.ord[p]
            if self.mlive[bb]:
                m = self.mlive[bb]
                return bb, (m & -m).bit_length() - 1
        return None

    # ---- maintenance
    def recompute_sb(self, from_sb):
        for s in range(from_sb, self.nsb()):
            idx = range(s * SB, min(self.nb, s * SB + SB))
            self.svis[s] = sum(popc(self.mvis[self.ord[i]]) for i in idx)
            self.scnt[s] = sum(self.bcnt[self.ord[i]] for i in idx)

    def split_block(self, b):
        if self.nb >= self.max_blocks:
            raise ModelError("capacity")
        b2 = self.nb
        for l in range(BLK // 2, BLK):
            v = self.items[b][l]
            self.items[b2][l - BLK // 2] = v
            self.blk[v] = b2
            self.slot[v] = l - BLK // 2
        p = self.opos[b] + 1
        for i in range(self.nb - 1, p - 1, -1):
            v = self.ord[i]
            self.ord[i + 1] = v
            self.opos[v] = i + 1
        self.mvis[b2] = self.mvis[b] >> 32
        self.mvis[b] &= 0xFFFFFFFF
        self.mlive[b2] = self.mlive[b] >> 32
        self.mlive[b] &= 0xFFFFFFFF
        self.bcnt[b2] = BLK // 2
        self.bcnt[b] = BLK // 2
        self.ord[p] = b2
        self.opos[b2] = p
        self.nb += 1
        self.recompute_sb((p - 1) // SB)
        return b2

    def insert_run(self, b, s, lv, k, ol, orr):
        for j in range(k):
            it = lv + j
            self.st[it] = 1
            self.aux[it] = ol if j == 0 else it - 1
            self.orr[it] = orr
        while k > 0:
            cnt = self.bcnt[b]
            if cnt == BLK:
                b2 = self.split_block(b)
                if s > BLK // 2:
                    b, s = b2, s - BLK // 2
                continue
            m = min(k, BLK - cnt)
            row = self.items[b]
            old = row[:]
            for l in range(s, cnt):
                row[l + m] = old[l]
                self.slot[old[l]] = l + m
            for l in range(s, s + m):
                it = lv + (l - s)
                row[l] = it
                self.slot[it] = l
                self.blk[it] = b
            low = 0 if s == 0 else (MASK64 >> (64 - s))
            ins = ((MASK64 if m == 64 else (1 << m) - 1) << s) & MASK64
            mv, ml = self.mvis[b], self.mlive[b]
            hv = 0 if m == 64 else (((mv & ~low) << m) & MASK64)
            hl = 0 if m == 64 else (((ml & ~low) << m) & MASK64)
            self.mvis[b] = (mv & low) | hv | ins
            self.mlive[b] = (ml & low) | hl | ins
            self.bcnt[b] = cnt + m
            sbi = self.opos[b] // SB
            self.svis[sbi] += m
            self.scnt[sbi] += m
            lv += m
            k -= m
            s += m

    def agent_of(self, lv):
        lo, hi = 0, len(self.aruns) // 3
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if self.aruns[3 * mid] <= lv:
                lo = mid
            else:
                hi = mid
        return self.aruns[3 * lo + 1], self.aruns[3 * lo + 2] + (lv - self.aruns[3 * lo])

    def rank_left(self, ol):
        return 0 if ol == ROOT_ID else self.rank_of(ol) + 1

    def rank_right(self, orr):
        return 1 << 64 if orr == END_ID else self.rank_of(orr)

    # ---- commands
    def do_insert(self, lv, k, pos):
        if pos == 0:
            ol = ROOT_ID
            cb, cs = self.ord[0], 0
        else:
            b, s = self.find_vis(pos - 1)
            ol = self.items[b][s]
            cb, cs = b, s + 1
        cb, cs = self.normalize(cb, cs)
        r = self.next_live(cb, cs)
        orr = self.items[r[0]][r[1]] if r else END_ID
        at_end = cs >= self.bcnt[cb]
        direct = (r == (cb, cs)) if r else at_end
        if not direct:
            my_l, my_r = self.rank_left(ol), self.rank_right(orr)
            nr, ns = self.agent_of(lv)
            scanning = False
            scan = (cb, cs)
            c = (cb, cs)
            while True:
                if c[1] >= self.bcnt[c[0]]:
                    break
                o = self.items[c[0]][c[1]]
                if o == orr:
                    break
                ol_o = self.rank_left(self.aux[o])
                if ol_o < my_l:
                    break
                if ol_o == my_l:
                    if self.orr[o] == orr:
                        r2, s2 = self.agent_of(o)
                        if nr < r2 or (nr == r2 and ns < s2):
                            break
                        scanning = False
                    else:
                        if self.rank_right(self.orr[o]) < my_r:
                            if not scanning:
                                scanning = True
                                scan = c
                        else:
                            scanning = False
                c = self.normalize(c[0], c[1] + 1)
            cb, cs = scan if scanning else c
        self.insert_run(cb, cs, lv, k, ol, orr)

    def do_delete(self, lv, n, pos, fwd):
        j0 = 0
        while j0 < n:
            b, s = self.find_vis(pos)
            vm = self.mvis[b] & (MASK64 << s) & MASK64
            take = min(popc(vm), n - j0)
            sel = 0
            r = 0
            for l in range(BLK):
                if (vm >> l) & 1:
                    if r < take:
                        item = self.items[b][l]
                        j = j0 + r
                        dlv = lv + j if fwd else lv + n - 1 - j
                        if (self.st[item] & 0x7F) != 1:
                            raise ModelError(f"delete of non-visible item {item}")
                        self.st[item] = DEL_BIT | 2
                        self.aux[dlv] = item
                        sel |= 1 << l
                    r += 1
            self.mvis[b] &= ~sel & MASK64
            self.svis[self.opos[b] // SB] -= take
            j0 += take

    def toggle(self, advance, is_del, lv, n):
        for j in range(n):
            v = lv + j
            item = self.aux[v] if is_del else v
            old = self.st[item]
            state = old & 0x7F
            b, s = self.blk[item], self.slot[item]
            bit = 1 << s
            sbi = self.opos[b] // SB
            if not is_del:
                if advance:
                    if state != 0:
                        raise ModelError(f"advance ins {item} state {state}")
                    self.st[item] = old | 1
                    self.mvis[b] |= bit
                    self.mlive[b] |= bit
                    self.svis[sbi] += 1
                else:
                    if state != 1:
                        raise ModelError(f"retreat ins {item} state {state}")
                    self.st[item] = old & DEL_BIT
                    self.mvis[b] &= ~bit
                    self.mlive[b] &= ~bit
                    self.svis[sbi] -= 1
            else:
                if advance:
                    if state == 0:
                        raise ModelError(f"advance del of NIY {item}")
                    self.st[item] = DEL_BIT | (state + 1)
                    if state == 1:
                        self.mvis[b] &= ~bit
                        self.svis[sbi] -= 1
                else:
                    if state < 2:
                        raise ModelError(f"retreat del {item} state {state}")
                    self.st[item] = (old & DEL_BIT) | (state - 1)
                    if state == 2:
                        self.mvis[b] |= bit
                        self.svis[sbi] += 1

    def run(self, check=None):
        for ci, (op, lv, ln, pos) in enumerate(self.cmds):
            code = op & 15
            if code == 0:
                self.do_insert(lv, ln, pos)
            elif code == 1:
                self.do_delete(lv, ln, pos, bool(op & 16))
            elif code == 2:
                self.toggle(True, False, lv, ln)
            elif code == 3:
                self.toggle(True, True, lv, ln)
            elif code == 4:
                self.toggle(False, False, lv, ln)
            elif code == 5:
                self.toggle(False, True, lv, ln)
            if check:
                check(self, ci)
        out = bytearray()
        for i in range(self.nb):
            b = self.ord[i]
            for l in range(self.bcnt[b]):
                it = self.items[b][l]
                if not (self.st[it] & DEL_BIT):
                    cb = self.cbyte[it]
                    c0 = self.content[cb]
                    n = 1 if c0 < 0x80 else 2 if (c0 & 0xE0) == 0xC0 else 3 if (c0 & 0xF0) == 0xE0 else 4
                    out += self.content[cb:cb + n]
        return bytes(out)


def check_invariants(d, ci=None):
    """Same structural invariants the kernel checks in DTGPU_DEBUG mode."""
    for i in range(d.nb):
        b = d.ord[i]
        if d.opos[b] != i:
            return 201
        cnt = d.bcnt[b]
        for l in range(64):
            if l < cnt:
                it = d.items[b][l]
                st = d.st[it] & 0x7F
                if ((d.mvis[b] >> l) & 1) != (1 if st == 1 else 0):
                    return 202
                if ((d.mlive[b] >> l) & 1) != (1 if st != 0 else 0):
                    return 202
                if d.blk[it] != b or d.slot[it] != l:
                    return 202
            elif ((d.mvis[b] | d.mlive[b]) >> l) & 1:
                return 202
    for s in range(d.nsb()):
        idx = range(s * SB, min(d.nb, s * SB + SB))
        if sum(popc(d.mvis[d.ord[i]]) for i in idx) != d.svis[s]:
            return 203
        if sum(d.bcnt[d.ord[i]] for i in idx) != d.scnt[s]:
            return 204
    return 0
