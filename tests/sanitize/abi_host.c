/*
 * abi_host.c — the device-free paths of the C ABI, for the host
 * AddressSanitizer + UndefinedBehaviorSanitizer build of the runtime
 * (tests/test_sanitize.py).  Without a GPU: build info, device creation failing
 * cleanly, shader lookup + reflection of every built-in program, pipeline
 * creation (no device: validation only) for valid and rejected state, the
 * validate_vertex_inputs error codes (pipeline.rs:134-143, 228-287), command
 * recording errors latched on a NULL device, and the collectives' host plans.
 * Prints "abi_host ok" and exits 0 when every expectation holds.
 */
#include <stdio.h>
#include <string.h>

#include "zenith_raster.h"

static int fails = 0;
#define EXPECT(c)                                                        \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                     \
        }                                                                \
    } while (0)

/* want == ZR_SUCCESS: the lookup succeeds; anything else: it fails */
static zr_shader* lookup(const char* path, const char* entry, uint32_t stage, zr_result want) {
    zr_shader* sh = NULL;
    const zr_result rc = zr_shader_lookup(NULL, path, entry, stage, &sh);
    EXPECT(want == ZR_SUCCESS ? rc == ZR_SUCCESS : rc != ZR_SUCCESS);
    if (rc == ZR_SUCCESS) {
        zr_shader_binding b[8];
        zr_vertex_input_attr a[8];
        const int32_t nb = zr_shader_bindings(sh, b, 8), na = zr_shader_vertex_inputs(sh, a, 8);
        EXPECT(nb >= 0 && nb <= 8 && na >= 0 && na <= 8);
        for (int32_t i = 0; i < nb; ++i) EXPECT(memchr(b[i].name, 0, sizeof b[i].name) != NULL);
        EXPECT(zr_shader_bindings(sh, NULL, 0) == nb);
    }
    return sh;
}

static zr_result pipeline(const zr_shader* vs, const zr_shader* fs, const zr_vertex_attribute* attrs, uint32_t nattrs,
                          uint32_t blend, uint32_t samples, zr_pipeline_error* err) {
    const zr_vertex_binding vb = {0, 24, 0};
    zr_color_attachment_desc cad;
    memset(&cad, 0, sizeof cad);
    cad.blend_enable = blend;
    cad.write_mask = 0xF;
    const int32_t fmt = 50; /* B8G8R8A8_SRGB */
    zr_graphic_pipeline_desc d;
    memset(&d, 0, sizeof d);
    d.vertex_shader = vs;
    d.fragment_shader = fs;
    d.vertex_binding_count = 1;
    d.vertex_bindings = &vb;
    d.vertex_attribute_count = nattrs;
    d.vertex_attributes = attrs;
    d.topology = 3; /* TRIANGLE_LIST */
    d.rasterization.line_width = 1.0f;
    d.samples = samples;
    d.color_attachment_count = 1;
    d.color_attachments = &cad;
    d.color_formats = &fmt;
    zr_pipeline* p = NULL;
    const zr_result rc = zr_pipeline_create(NULL, &d, &p, err);
    if (rc == ZR_SUCCESS) zr_pipeline_destroy(p);
    return rc;
}

int main(void) {
    EXPECT(strstr(zr_build_info(), "gfx950") != NULL);
    zr_device* dev = NULL;
    const zr_result drc = zr_device_create(0, &dev);
    if (drc == ZR_SUCCESS) zr_device_destroy(dev); /* a GPU is present: nothing more to check here */
    EXPECT(zr_last_error_message() != NULL);

    const char* progs[] = {"content/shaders/triangle.slang", "content/shaders/flat_color.slang",
                           "content/shaders/blinn_phong.slang", "content/shaders/mesh.slang"};
    zr_shader* sh[4][2];
    for (int i = 0; i < 4; ++i) {
        sh[i][0] = lookup(progs[i], "vsmain", ZR_SHADER_STAGE_VERTEX, ZR_SUCCESS);
        sh[i][1] = lookup(progs[i], "psmain", ZR_SHADER_STAGE_FRAGMENT, ZR_SUCCESS);
    }
    lookup("content/shaders/missing.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, ZR_ERROR_SHADER_NOT_FOUND);
    lookup("content/shaders/triangle.slang", "psmain", ZR_SHADER_STAGE_VERTEX, ZR_ERROR_SHADER_NOT_FOUND);

    const zr_vertex_attribute ok[2] = {{0, 0, 106, 0}, {1, 0, 106, 12}};       /* R32G32B32_SFLOAT x2 */
    const zr_vertex_attribute miss[1] = {{0, 0, 106, 0}};
    const zr_vertex_attribute mism[2] = {{0, 0, 106, 0}, {1, 0, 103, 12}};     /* R32G32_SFLOAT */
    const zr_vertex_attribute extra[3] = {{0, 0, 106, 0}, {1, 0, 106, 12}, {2, 0, 106, 24}};
    const zr_vertex_attribute dup[3] = {{0, 0, 106, 0}, {0, 0, 100, 0}, {1, 0, 106, 12}};
    zr_pipeline_error err;
    EXPECT(pipeline(sh[0][0], sh[0][1], ok, 2, 0, 1, &err) == ZR_SUCCESS);
    EXPECT(pipeline(sh[0][0], sh[0][1], miss, 1, 0, 1, &err) == ZR_ERROR_MISSING_VERTEX_ATTRIBUTE && err.location == 1);
    EXPECT(pipeline(sh[0][0], sh[0][1], mism, 2, 0, 1, &err) == ZR_ERROR_VERTEX_ATTRIBUTE_FORMAT_MISMATCH);
    EXPECT(pipeline(sh[0][0], sh[0][1], extra, 3, 0, 1, &err) == ZR_ERROR_UNEXPECTED_VERTEX_ATTRIBUTE && err.location == 2);
    EXPECT(pipeline(sh[0][0], sh[0][1], dup, 3, 0, 1, &err) == ZR_ERROR_DUPLICATE_VERTEX_ATTRIBUTE_LOCATION);
    EXPECT(pipeline(NULL, sh[0][1], ok, 2, 0, 1, &err) == ZR_ERROR_MISSING_VERTEX_SHADER);
    EXPECT(pipeline(sh[0][0], sh[0][1], ok, 2, 1, 1, NULL) == ZR_ERROR_FEATURE_NOT_PRESENT); /* blending */
    EXPECT(pipeline(sh[0][0], sh[0][1], ok, 2, 0, 4, NULL) == ZR_ERROR_FEATURE_NOT_PRESENT); /* MSAA */
    EXPECT(pipeline(sh[0][0], sh[1][1], ok, 2, 0, 1, NULL) == ZR_ERROR_FEATURE_NOT_PRESENT); /* mixed programs */

    /* recording with a NULL command list is a no-op */
    zr_cmd_set_tile_shard(NULL, 0, 1);
    zr_cmd_set_route_capacity(NULL, 0);
    zr_cmd_push_constants(NULL, NULL, 0, 0, 0, NULL);

    /* push constants (command.rs:180-185) on a device-less list: host validation */
    {
        zr_shader *mvs = NULL, *mps = NULL;
        EXPECT(zr_shader_lookup(NULL, "content/shaders/mesh_push.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, &mvs) == 0);
        EXPECT(zr_shader_lookup(NULL, "content/shaders/mesh_push.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, &mps) == 0);
        EXPECT(zr_shader_push_constant_size(mvs) == 64 && zr_shader_push_constant_size(mps) == 0);
        const zr_vertex_binding mvb = {0, 32, 0};
        const zr_vertex_attribute mat[3] = {{0, 0, ZR_FORMAT_R32G32B32_SFLOAT, 0}, {1, 0, ZR_FORMAT_R32G32B32_SFLOAT, 12},
                                            {2, 0, ZR_FORMAT_R32G32_SFLOAT, 24}};
        zr_graphic_pipeline_desc d;
        memset(&d, 0, sizeof d);
        d.vertex_shader = mvs;
        d.fragment_shader = mps;
        d.vertex_binding_count = 1;
        d.vertex_bindings = &mvb;
        d.vertex_attribute_count = 3;
        d.vertex_attributes = mat;
        d.topology = 3;
        d.samples = 1;
        zr_pipeline* mp = NULL;
        EXPECT(zr_pipeline_create(NULL, &d, &mp, NULL) == ZR_SUCCESS);
        zr_push_constant_range rg[2];
        EXPECT(zr_pipeline_push_constant_ranges(mp, rg, 2) == 1 && rg[0].stage_flags == ZR_SHADER_STAGE_ALL_GRAPHICS &&
               rg[0].offset == 0 && rg[0].size == 64);
        const zr_push_constant_range short_range = {ZR_SHADER_STAGE_VERTEX, 0, 32};
        d.push_constant_range_count = 1;
        d.push_constant_ranges = &short_range;
        zr_pipeline* bad = NULL;
        EXPECT(zr_pipeline_create(NULL, &d, &bad, NULL) == ZR_ERROR_VALIDATION_FAILED && bad == NULL);
        float view[16];
        for (int i = 0; i < 16; ++i) view[i] = (float)i;
        zr_cmd* cmd = NULL;
        EXPECT(zr_cmd_create(NULL, &cmd) == ZR_SUCCESS && cmd != NULL);
        EXPECT(zr_cmd_begin(cmd) == ZR_SUCCESS);
        zr_cmd_push_constants(cmd, mp, ZR_SHADER_STAGE_ALL_GRAPHICS, 0, 64, view);
        zr_cmd_push_constants(cmd, mp, ZR_SHADER_STAGE_ALL_GRAPHICS, 16, 16, view);
        EXPECT(zr_cmd_end(cmd) == ZR_SUCCESS);
        EXPECT(zr_submit((zr_device*)view, cmd, NULL) == ZR_ERROR_VALIDATION_FAILED); /* not its device */
        EXPECT(zr_cmd_begin(cmd) == ZR_SUCCESS);
        zr_cmd_push_constants(cmd, mp, ZR_SHADER_STAGE_VERTEX, 0, 64, view); /* misses the range's stages */
        EXPECT(zr_cmd_end(cmd) == ZR_ERROR_VALIDATION_FAILED);
        EXPECT(zr_cmd_begin(cmd) == ZR_SUCCESS);
        zr_cmd_push_constants(cmd, mp, ZR_SHADER_STAGE_ALL_GRAPHICS, 60, 8, view); /* past the range */
        EXPECT(zr_cmd_end(cmd) == ZR_ERROR_VALIDATION_FAILED);
        zr_cmd_destroy(cmd);
        zr_pipeline_destroy(mp);
        zr_shader_destroy(mvs);
        zr_shader_destroy(mps);
    }

    /* the collectives' host plans (tests/test_abi.py checks their content) */
    zr_transfer_op ops[80];
    for (int32_t g = 1; g <= 8; ++g)
        for (int32_t r = 0; r < g; ++r) {
            const int32_t n = zr_gather_plan(1920, 1080, 4, g, r, 0, ops, 80);
            EXPECT(n >= 0 && n <= 80 && zr_gather_plan(1920, 1080, 4, g, r, 0, NULL, 0) == n);
            EXPECT(zr_exchange_plan(g, r, 16 + 48 * 100, ops, 80) == 2 * g);
            EXPECT(zr_gather_plan(1920, 1080, 4, g, r, 0, ops, 1) == n); /* capacity 1: count only past it */
        }
    EXPECT(zr_exchange_plan(33, 0, 64, ops, 80) == -1);

    for (int i = 0; i < 4; ++i) {
        zr_shader_destroy(sh[i][0]);
        zr_shader_destroy(sh[i][1]);
    }
    if (fails) return 1;
    printf("abi_host ok\n");
    return 0;
}
