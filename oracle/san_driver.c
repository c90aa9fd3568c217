/*
 * san_driver.c — runs one oracle draw from a scene file, for the host
 * AddressSanitizer + UndefinedBehaviorSanitizer build of the oracle
 * (TEST INFRASTRUCTURE ONLY: tests/test_sanitize.py builds and runs it).
 *
 * Scene file (little-endian, written by tests/test_sanitize.py from the same
 * ctypes structures oracle.py passes to the library):
 *   u32 magic 'ZRSB', u32 nthreads
 *   zro_draw_state, zro_draw_cmd          (raw structs)
 *   u32 width, height; i32 color_format; u32 has_depth; i32 render_area[4];
 *   f32 clear_color[4]; f32 clear_depth; u32 tile_size; u32 stride; u32 attr_count;
 *   u32 attr_offset[4]; u32 attr_size[4]; i32 index_type; u64 vertex_bytes; u64 index_bytes
 *   vertex bytes, index bytes (index_bytes = 0: non-indexed)
 * Every buffer is a heap block of exactly its size, so an access one byte past
 * any of them is reported.  Writes colour then depth to argv[2].
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zr_oracle.h"

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s scene.bin out.bin\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint32_t magic = 0, nthreads = 1;
    zro_draw_state st;
    zro_draw_cmd cmd;
    uint32_t w, h, has_depth, tile, stride, nattr, aoff[4], asz[4];
    int32_t fmt, ra[4], itype;
    float clear[4], clear_depth;
    uint64_t vbytes, ibytes;
    if (rd(f, &magic, 4) || magic != 0x4253525Au || rd(f, &nthreads, 4) || rd(f, &st, sizeof st) ||
        rd(f, &cmd, sizeof cmd) || rd(f, &w, 4) || rd(f, &h, 4) || rd(f, &fmt, 4) || rd(f, &has_depth, 4) ||
        rd(f, ra, 16) || rd(f, clear, 16) || rd(f, &clear_depth, 4) || rd(f, &tile, 4) || rd(f, &stride, 4) ||
        rd(f, &nattr, 4) || rd(f, aoff, 16) || rd(f, asz, 16) || rd(f, &itype, 4) || rd(f, &vbytes, 8) ||
        rd(f, &ibytes, 8)) {
        fprintf(stderr, "bad scene file\n");
        return 2;
    }
    uint8_t* vb = malloc(vbytes ? vbytes : 1);
    uint8_t* ib = ibytes ? malloc(ibytes) : NULL;
    if (!vb || (ibytes && !ib) || rd(f, vb, vbytes) || (ibytes && rd(f, ib, ibytes))) return 2;
    fclose(f);
    const uint32_t bpp = zro_format_bpp(fmt);
    uint8_t* color = calloc((size_t)w * h, bpp);
    float* depth = has_depth ? malloc((size_t)w * h * sizeof(float)) : NULL;
    if (!color || (has_depth && !depth)) return 2;
    if (depth)
        for (size_t i = 0; i < (size_t)w * h; ++i) depth[i] = __builtin_nanf(""); /* rows a shard does not own stay NaN */
    zro_target t = {w, h, fmt, color, depth};
    zro_clear(&t, ra, clear, 1, clear_depth, depth != NULL, tile, st.shard_rank, st.shard_count);
    zro_vertex_input vi;
    memset(&vi, 0, sizeof vi);
    vi.vertex_data = vb;
    vi.vertex_bytes = vbytes;
    vi.stride = stride;
    vi.attr_count = nattr;
    memcpy(vi.attr_offset, aoff, sizeof aoff);
    memcpy(vi.attr_size, asz, sizeof asz);
    vi.index_data = ib;
    vi.index_bytes = ibytes;
    vi.index_type = itype;
    zro_stats stats;
    const int rc = zro_draw(&t, &st, &vi, &cmd, (int)nthreads, &stats);
    if (rc != 0) {
        fprintf(stderr, "zro_draw failed: %d\n", rc);
        return 1;
    }
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 2;
    fwrite(color, 1, (size_t)w * h * bpp, o);
    if (depth) fwrite(depth, sizeof(float), (size_t)w * h, o);
    fclose(o);
    free(vb);
    free(ib);
    free(color);
    free(depth);
    printf("triangles_setup %llu\n", (unsigned long long)stats.triangles_setup);
    return 0;
}
