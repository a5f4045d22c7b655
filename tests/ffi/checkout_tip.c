/* Links lib/libdtgpu.a (the static library a Rust `build.rs` would link, see
 * crates/dtgpu-sys) from plain C and runs the drop-in path on one .dt file:
 *   ListOpLog::load_from(bytes)?.checkout_tip().content()   (decode_oplog.rs:447, oplog.rs:38)
 * and, through the batch entry, many of them at once (dtgpu_batch_checkout).
 * Usage: checkout_tip FILE.dt OUT.txt   -> writes the text, prints "len hash". */
#include <stdio.h>
#include <stdlib.h>
#include "dtgpu.h"

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s FILE.dt OUT.txt\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror("open"); return 2; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *bytes = malloc((size_t)n);
    if (fread(bytes, 1, (size_t)n, f) != (size_t)n) { fclose(f); return 2; }
    fclose(f);
    dtgpu_oplog *o = NULL;
    dtgpu_status s = dtgpu_oplog_load(bytes, (size_t)n, 0, &o);
    if (s != DTGPU_OK) { fprintf(stderr, "load: %d\n", (int)s); return 1; }
    size_t len = 0;
    s = dtgpu_checkout_tip(o, NULL, 0, &len);                 /* length query */
    if (s != DTGPU_OK) { fprintf(stderr, "checkout (size): %d\n", (int)s); return 1; }
    uint8_t *text = malloc(len + 1);
    s = dtgpu_checkout_tip(o, text, len, &len);
    if (s != DTGPU_OK) { fprintf(stderr, "checkout: %d\n", (int)s); return 1; }
    FILE *g = fopen(argv[2], "wb");
    if (!g || fwrite(text, 1, len, g) != len) { perror("write"); return 2; }
    fclose(g);
    /* batch entry: 4 copies, every one must match the single checkout */
    const uint8_t *docs[4] = {bytes, bytes, bytes, bytes};
    size_t lens[4] = {(size_t)n, (size_t)n, (size_t)n, (size_t)n};
    dtgpu_doc_result res[4];
    s = dtgpu_batch_checkout(docs, lens, 4, NULL, res);
    if (s != DTGPU_OK) { fprintf(stderr, "batch: %d\n", (int)s); return 1; }
    const uint64_t h = dtgpu_text_hash(text, len);
    for (int i = 0; i < 4; i++)
        if (res[i].status != 0 || res[i].text_len != len || res[i].text_hash != h) {
            fprintf(stderr, "batch doc %d differs\n", i);
            return 1;
        }
    printf("%zu %llu\n", len, (unsigned long long)h);
    dtgpu_oplog_free(o);
    free(text);
    free(bytes);
    return 0;
}
