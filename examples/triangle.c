/*
 * triangle.c — zenith's examples/triangle.rs frame, driven through the C ABI.
 *
 * The same call sequence TriangleRenderer::render_to records on zenith-rhi
 * (zenith-renderer/src/triangle.rs:28-178), one call per reference call:
 * buffers + upload, Shader::from_file x2, GraphicShaderInput + pipeline state,
 * begin_rendering, bind_pipeline, Time uniform, set_viewport/scissor,
 * bind_vertex/index_buffer, draw_indexed(3,1,0,0,0), end_rendering, submit.
 * Writes the BGRA8 frame as raw bytes to argv[1] (default triangle.bgra).
 *
 *   gcc -O2 -Iinclude examples/triangle.c -Lzenith_amd/lib -lzenith_raster \
 *       -Wl,-rpath,$PWD/zenith_amd/lib -o triangle_c
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zenith_raster.h"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        zr_result rc_ = (x);                                                              \
        if (rc_ != ZR_SUCCESS) {                                                          \
            fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, (int)rc_,   \
                    zr_last_error_message());                                             \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

int main(int argc, char** argv) {
    const char* out_path = argc > 1 ? argv[1] : "triangle.bgra";
    const uint32_t W = 640, H = 480;
    const float elapsed = argc > 2 ? (float)atof(argv[2]) : 0.0f;

    zr_device* dev = NULL;
    CHECK(zr_device_create(0, &dev));

    /* triangle.rs:28-49 — vertices {position, color}, u16 indices, uploaded once */
    const float vertices[3][6] = {{0.0f, 0.5f, 0.0f, 1.0f, 0.0f, 0.0f},
                                  {-0.5f, -0.5f, 0.0f, 0.0f, 1.0f, 0.0f},
                                  {0.5f, -0.5f, 0.0f, 0.0f, 0.0f, 1.0f}};
    const uint16_t indices[3] = {0, 1, 2};
    zr_buffer *vb = NULL, *ib = NULL, *tb = NULL;
    zr_buffer_desc vd = {"triangle.vertex", sizeof vertices, ZR_BUFFER_USAGE_VERTEX | ZR_BUFFER_USAGE_TRANSFER_DST,
                         ZR_MEMORY_DEVICE_LOCAL};
    zr_buffer_desc id = {"triangle.index", sizeof indices, ZR_BUFFER_USAGE_INDEX | ZR_BUFFER_USAGE_TRANSFER_DST,
                         ZR_MEMORY_DEVICE_LOCAL};
    zr_buffer_desc td = {"triangle.time", 4, ZR_BUFFER_USAGE_UNIFORM, ZR_MEMORY_HOST_VISIBLE | ZR_MEMORY_HOST_COHERENT};
    CHECK(zr_buffer_create(dev, &vd, &vb));
    CHECK(zr_buffer_create(dev, &id, &ib));
    CHECK(zr_buffer_create(dev, &td, &tb));
    CHECK(zr_buffer_write(vb, 0, vertices, sizeof vertices));
    CHECK(zr_buffer_write(ib, 0, indices, sizeof indices));

    /* triangle.rs:52-66 */
    zr_shader *vs = NULL, *ps = NULL;
    CHECK(zr_shader_lookup(dev, "content/shaders/triangle.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, &vs));
    CHECK(zr_shader_lookup(dev, "content/shaders/triangle.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, &ps));

    /* triangle.rs:104-122 — vertex layout derived from Vertex, clear colour, cull NONE */
    const zr_vertex_binding binding = {0, 24, 0};
    const zr_vertex_attribute attrs[2] = {{0, 0, ZR_FORMAT_R32G32B32_SFLOAT, 0},
                                          {1, 0, ZR_FORMAT_R32G32B32_SFLOAT, 12}};
    zr_color_attachment_desc color_desc;
    memset(&color_desc, 0, sizeof color_desc);
    color_desc.write_mask = 0xF;
    color_desc.load_op = ZR_ATTACHMENT_LOAD_OP_CLEAR;
    color_desc.store_op = ZR_ATTACHMENT_STORE_OP_STORE;
    color_desc.clear_value[0] = color_desc.clear_value[1] = color_desc.clear_value[2] = 0.1f;
    color_desc.clear_value[3] = 1.0f;
    const int32_t color_format = ZR_FORMAT_B8G8R8A8_SRGB;
    zr_graphic_pipeline_desc pd;
    memset(&pd, 0, sizeof pd);
    pd.vertex_shader = vs;
    pd.fragment_shader = ps;
    pd.vertex_binding_count = 1;
    pd.vertex_bindings = &binding;
    pd.vertex_attribute_count = 2;
    pd.vertex_attributes = attrs;
    pd.topology = 3; /* TRIANGLE_LIST */
    pd.rasterization.polygon_mode = 0;
    pd.rasterization.cull_mode = 0; /* NONE (triangle.rs:116) */
    pd.rasterization.front_face = 0;
    pd.rasterization.line_width = 1.0f;
    pd.samples = 1;
    pd.color_attachment_count = 1;
    pd.color_attachments = &color_desc;
    pd.color_formats = &color_format;
    zr_pipeline* pipe = NULL;
    zr_pipeline_error perr;
    CHECK(zr_pipeline_create(dev, &pd, &pipe, &perr));

    zr_texture* target = NULL;
    zr_texture_desc tdesc = {"swapchain", W, H, color_format, 0};
    CHECK(zr_texture_create(dev, &tdesc, &target));

    /* triangle.rs:127-178 — the graphic node's job */
    CHECK(zr_buffer_write(tb, 0, &elapsed, 4));
    zr_cmd* cmd = NULL;
    CHECK(zr_cmd_create(dev, &cmd));
    CHECK(zr_cmd_begin(cmd));
    zr_rendering_attachment ca;
    memset(&ca, 0, sizeof ca);
    ca.texture = target;
    ca.load_op = ZR_ATTACHMENT_LOAD_OP_CLEAR;
    ca.store_op = ZR_ATTACHMENT_STORE_OP_STORE;
    memcpy(ca.clear_value, color_desc.clear_value, sizeof ca.clear_value);
    zr_rendering_info ri = {{0, 0, W, H}, 1, &ca, NULL};
    zr_cmd_begin_rendering(cmd, &ri);
    zr_cmd_bind_pipeline(cmd, pipe);
    CHECK(zr_cmd_bind_uniform_by_name(cmd, pipe, "Time", tb, 0, 4));
    const zr_viewport vp = {0.0f, 0.0f, (float)W, (float)H, 0.0f, 1.0f};
    const zr_rect2d sc = {0, 0, W, H};
    zr_cmd_set_viewport(cmd, 0, 1, &vp);
    zr_cmd_set_scissor(cmd, 0, 1, &sc);
    const zr_buffer* vbs[1] = {vb};
    const uint64_t offs[1] = {0};
    zr_cmd_bind_vertex_buffers(cmd, 0, 1, vbs, offs);
    zr_cmd_bind_index_buffer(cmd, ib, 0, ZR_INDEX_TYPE_UINT16);
    zr_cmd_draw_indexed(cmd, 3, 1, 0, 0, 0);
    zr_cmd_end_rendering(cmd);
    CHECK(zr_cmd_end(cmd));
    CHECK(zr_submit_and_wait(dev, cmd));

    /* headless "present": read the frame back */
    const size_t bytes = (size_t)W * H * 4;
    unsigned char* img = (unsigned char*)malloc(bytes);
    CHECK(zr_texture_read(target, img, bytes));
    FILE* f = fopen(out_path, "wb");
    if (!f || fwrite(img, 1, bytes, f) != bytes) {
        fprintf(stderr, "cannot write %s\n", out_path);
        return 1;
    }
    fclose(f);
    size_t covered = 0;
    for (size_t i = 0; i < (size_t)W * H; ++i)
        covered += !(img[4 * i] == 89 && img[4 * i + 1] == 89 && img[4 * i + 2] == 89);
    printf("triangle: %zu covered pixels -> %s\n", covered, out_path);
    free(img);

    zr_cmd_destroy(cmd);
    zr_texture_destroy(target);
    zr_pipeline_destroy(pipe);
    zr_shader_destroy(vs);
    zr_shader_destroy(ps);
    zr_buffer_destroy(tb);
    zr_buffer_destroy(ib);
    zr_buffer_destroy(vb);
    zr_device_destroy(dev);
    return 0;
}
