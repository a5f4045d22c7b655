// host_fuzz.cpp -- the product's host decoder / encoder / planner (dt_host.cpp, dt_encode.cpp)
// under AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_host_sanitizers.py builds and
// runs it; CPU only).  The fault-injection pattern follows the reference's encoding tests
// (src/list/encoding/tests.rs:180-235): every single-byte corruption of a small `.dt` file must
// decode to a status, never a crash or an out-of-bounds access; the benchmark files are decoded,
// planned, re-encoded and decoded again, merged into themselves and into their own prefixes with
// decode_and_add, and corrupted at a stride.
//   host_fuzz FILE... [BASE+PATCH...]   (every argument a `.dt` file, or a base and a patch
//   that decode_and_add merges into it, corrupted; files under 4 KiB get every corruption,
//   bigger ones about 200 positions, each decoded and, when it still decodes, planned)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "dt_host.hpp"

using namespace dtgpu;

static std::vector<uint8_t> read_file(const char *path) {
    std::vector<uint8_t> d;
    FILE *f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    uint8_t buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + n);
    fclose(f);
    return d;
}

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); fails++; } } while (0)

// decode -> plan -> plan input (files up to 64 KiB); returns the decode status
static Status exercise(const std::vector<uint8_t> &d, bool ignore_crc) {
    HostOpLog o;
    const Status s = decode_dt(d.data(), d.size(), ignore_crc, o);
    if (s != OK || d.size() > 65536) return s;   // big files: the decoder only
    Plan p;
    (void)build_plan(o, p);
    PlanInput pi;
    (void)build_plan_input(o, pi);
    return s;
}

int main(int argc, char **argv) {
    size_t corruptions = 0;
    for (int a = 1; a < argc; a++) {
        const std::string arg = argv[a];
        if (arg.find('+') != std::string::npos) {   // a patch merged into its base, then corrupted
            const std::vector<uint8_t> base = read_file(arg.substr(0, arg.find('+')).c_str());
            const std::vector<uint8_t> patch = read_file(arg.substr(arg.find('+') + 1).c_str());
            HostOpLog o;
            std::vector<uint64_t> ff;
            CHECK(decode_and_add(base.data(), base.size(), false, o, ff) == OK, "%s: base", argv[a]);
            HostOpLog m = o;
            CHECK(decode_and_add(patch.data(), patch.size(), false, m, ff) == OK, "%s: patch", argv[a]);
            for (size_t i = 0; i < patch.size(); i++) {
                for (uint8_t x : {uint8_t(0x01), uint8_t(0x40), uint8_t(0x80), uint8_t(0xFF)}) {
                    std::vector<uint8_t> c = patch;
                    c[i] ^= x;
                    for (bool ic : {false, true}) {
                        HostOpLog e = o;
                        if (decode_and_add(c.data(), c.size(), ic, e, ff) != OK)
                            CHECK(e.n_lv == o.n_lv, "%s: failed patch changed the oplog", argv[a]);
                        corruptions++;
                    }
                }
            }
            printf("%s: %llu LVs ok\n", argv[a], (unsigned long long)m.n_lv);
            continue;
        }
        const std::vector<uint8_t> d = read_file(argv[a]);
        HostOpLog o;
        const Status s = decode_dt(d.data(), d.size(), false, o);
        CHECK(s == OK, "%s: decode status %d", argv[a], int(s));
        if (s != OK) continue;
        Plan p;
        CHECK(build_plan(o, p) == OK, "%s: build_plan failed", argv[a]);
        PlanInput pi;
        (void)build_plan_input(o, pi);
        // encode from ROOT (compressed and not), decode again: same LVs and version
        for (bool lz4 : {true, false}) {
            std::vector<uint8_t> enc;
            CHECK(encode_dt(o, {}, true, lz4, nullptr, enc) == OK, "%s: encode failed", argv[a]);
            HostOpLog o2;
            CHECK(decode_dt(enc.data(), enc.size(), false, o2) == OK, "%s: re-decode failed", argv[a]);
            // (LVs are local: the encoder's walk order may renumber concurrent entries, so the
            // frontier is compared by size; the texts' equality is test_encoder.py's job)
            CHECK(o2.n_lv == o.n_lv && o2.version.size() == o.version.size(),
                  "%s: round trip differs", argv[a]);
        }
        // decode_and_add: into an empty oplog, into itself (a no-op), and a prefix's patch
        {
            HostOpLog e;
            std::vector<uint64_t> ff;
            CHECK(decode_and_add(d.data(), d.size(), false, e, ff) == OK && e.n_lv == o.n_lv, "%s: add to empty", argv[a]);
            CHECK(decode_and_add(d.data(), d.size(), false, e, ff) == OK && e.n_lv == o.n_lv, "%s: add to itself", argv[a]);
        }
        if (o.n_lv > 2) {   // the history up to the middle entry, then the rest as a patch
            const uint64_t mid = o.graph.entries[o.graph.entries.size() / 2].end - 1;
            std::vector<uint8_t> all, patch;
            CHECK(encode_dt(o, {}, true, true, nullptr, all) == OK, "%s: encode", argv[a]);
            CHECK(encode_dt(o, {mid}, true, true, nullptr, patch) == OK, "%s: encode_from", argv[a]);
            HostOpLog e;
            std::vector<uint64_t> ff;
            CHECK(decode_and_add(all.data(), all.size(), false, e, ff) == OK, "%s: add all", argv[a]);
            CHECK(decode_and_add(patch.data(), patch.size(), false, e, ff) == OK && e.n_lv == o.n_lv,
                  "%s: add the patch again", argv[a]);
            // corrupted patches into the merged oplog: a status, and the oplog unchanged on error
            const size_t stride = patch.size() < 4096 ? 1 : patch.size() / 64;
            for (size_t i = 0; i < patch.size(); i += stride) {
                for (uint8_t x : {uint8_t(0x01), uint8_t(0x80), uint8_t(0xFF)}) {
                    std::vector<uint8_t> c = patch;
                    c[i] ^= x;
                    HostOpLog e2 = e;
                    std::vector<uint64_t> ff2;
                    if (decode_and_add(c.data(), c.size(), true, e2, ff2) != OK)
                        CHECK(e2.n_lv == e.n_lv, "%s: failed patch changed the oplog", argv[a]);
                    corruptions++;
                }
            }
        }
        // corruptions of the file itself (CRC checked and ignored)
        const size_t stride = d.size() < 4096 ? 1 : d.size() / (d.size() > 65536 ? 40 : 200);
        for (size_t i = 0; i < d.size(); i += stride) {
            for (uint8_t x : {uint8_t(0x01), uint8_t(0x40), uint8_t(0xFF)}) {
                std::vector<uint8_t> c = d;
                c[i] ^= x;
                (void)exercise(c, false);
                (void)exercise(c, true);
                corruptions += 2;
            }
        }
        // truncations
        for (size_t n = 0; n < d.size(); n += (d.size() < 4096 ? 1 : d.size() / 64)) {
            std::vector<uint8_t> c(d.begin(), d.begin() + n);
            (void)exercise(c, true);
            corruptions++;
        }
        // LZ4 round trip of the inserted content
        {
            std::vector<uint8_t> z, back(o.ins_content.size());
            lz4_block_compress(o.ins_content.data(), o.ins_content.size(), z);
            CHECK(lz4_block_decompress(z.data(), z.size(), back.data(), back.size()) && back == o.ins_content,
                  "%s: lz4 round trip", argv[a]);
        }
        printf("%s: %llu LVs ok\n", argv[a], (unsigned long long)o.n_lv);
    }
    printf("corrupted inputs decoded: %zu, failures: %d\n", corruptions, fails);
    return fails ? 1 : 0;
}
