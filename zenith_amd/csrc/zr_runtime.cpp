// zr_runtime.cpp — host side of libzenith_raster: the C ABI in include/zenith_raster.h.
//
// Objects mirror zenith-rhi's (RenderDevice, Buffer, Texture, Shader, pipeline,
// CommandEncoder, Fence); command buffers record like vkCmd* and are executed at
// zr_submit by walking the recorded state machine and launching the HIP passes
// of zr_kernels.hip on the device's stream.  No CPU fallback:
// every draw runs the HIP kernels or returns an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "zenith_raster.h"
#include "zr_internal.h"
#include "zr_rccl.h"
#include "zr_shading.h"

using namespace zr;

namespace {

thread_local std::string g_last_error = "";

zr_result fail(zr_result code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define ZR_HIP(expr)                                                                              \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) {                                                                   \
            return fail(_e == hipErrorOutOfMemory ? ZR_ERROR_OUT_OF_DEVICE_MEMORY : ZR_ERROR_DEVICE_LOST, \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                       \
        }                                                                                         \
    } while (0)

// ------------------------------------------------------------ shader registry

struct ShaderEntry {
    const char* file;
    const char* entry;
    uint32_t stage;
    int32_t program;
    int nbind;
    zr_shader_binding bind[1];
    int ninputs;
    zr_vertex_input_attr inputs[4];
    uint32_t push_size;  // ShaderReflection::push_constant_size (shader.rs:214)
};

// Built-in stage variants.  triangle.slang is the reference's
// (content/shaders/triangle.slang:3-8 inputs, :27-32 "Time" at set 0 / binding 0);
// flat_color / blinn_phong are this repo's (content/shaders/).
const ShaderEntry kShaders[] = {
    {"triangle.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, kProgTriangle, 0, {},
     2, {{0, ZR_FORMAT_R32G32B32_SFLOAT}, {1, ZR_FORMAT_R32G32B32_SFLOAT}}},
    {"triangle.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, kProgTriangle, 1,
     {{"Time", 0, 0, ZR_DESCRIPTOR_TYPE_UNIFORM_BUFFER, 1, ZR_SHADER_STAGE_FRAGMENT}}, 0, {}},
    {"flat_color.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, kProgFlat, 0, {},
     2, {{0, ZR_FORMAT_R32G32B32_SFLOAT}, {1, ZR_FORMAT_R32G32B32_SFLOAT}}},
    {"flat_color.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, kProgFlat, 0, {}, 0, {}},
    {"blinn_phong.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, kProgBlinn, 0, {},
     3, {{0, ZR_FORMAT_R32G32B32_SFLOAT}, {1, ZR_FORMAT_R32G32B32_SFLOAT}, {2, ZR_FORMAT_R32G32B32_SFLOAT}}},
    {"blinn_phong.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, kProgBlinn, 0, {}, 0, {}},
    // mesh.slang: camera program over zenith-asset's Vertex
    // {position, normal, uv} (zenith-asset/src/render.rs:12-16); View = view_proj
    {"mesh.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, kProgMesh, 1,
     {{"View", 0, 0, ZR_DESCRIPTOR_TYPE_UNIFORM_BUFFER, 1, ZR_SHADER_STAGE_VERTEX}},
     3, {{0, ZR_FORMAT_R32G32B32_SFLOAT}, {1, ZR_FORMAT_R32G32B32_SFLOAT}, {2, ZR_FORMAT_R32G32_SFLOAT}}},
    {"mesh.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, kProgMesh, 0, {}, 0, {}},
    // mesh_push.slang: the same program with view_proj in a 64-B push-constant
    // block (CommandEncoder::push_constants, command.rs:180-185) instead of View
    {"mesh_push.slang", "vsmain", ZR_SHADER_STAGE_VERTEX, kProgMesh, 0, {},
     3, {{0, ZR_FORMAT_R32G32B32_SFLOAT}, {1, ZR_FORMAT_R32G32B32_SFLOAT}, {2, ZR_FORMAT_R32G32_SFLOAT}}, 64},
    {"mesh_push.slang", "psmain", ZR_SHADER_STAGE_FRAGMENT, kProgMesh, 0, {}, 0, {}},
};

std::string basename_of(const char* path) {
    std::string p(path ? path : "");
    const size_t s = p.find_last_of("/\\");
    return s == std::string::npos ? p : p.substr(s + 1);
}

}  // namespace

// ------------------------------------------------------------------ objects

struct zr_shader_t {
    int32_t program;
    uint32_t stage;
    std::string file, entry;
    std::vector<zr_shader_binding> bindings;
    std::vector<zr_vertex_input_attr> inputs;
    uint32_t push_constant_size = 0;
};

struct zr_buffer_t {
    zr_device* dev;
    void* ptr;
    uint64_t size;
    bool external;
    std::string name;
};

struct zr_texture_t {
    zr_device* dev;
    void* ptr;
    uint32_t width, height;
    int32_t format;
    uint32_t bpp;
    bool external;
    std::string name;
    // zr_device_gather_tile_rows: the gather that last read this texture (the
    // next render pass writing it waits for it on the device stream)
    hipEvent_t gather_done = nullptr;
    bool gather_pending = false;
};

struct zr_pipeline_t {
    int32_t program;
    bool has_fs;
    uint32_t stride;
    uint32_t nattr;
    uint32_t attr_offset[4];
    uint32_t attr_size[4];
    std::vector<zr_shader_binding> bindings;  // merged reflection
    uint32_t push_size = 0;                   // merged push_constant_size (shader.rs:224-228)
    std::vector<zr_push_constant_range> push_ranges;  // the layout's (pipeline.rs:112-128)
    bool view_push = false;                   // mesh program reading view_proj from push constants
    uint32_t cull_mode;
    int32_t front_face;
    bool has_depth_state;
    zr_depth_stencil_desc ds;
    uint32_t color_count;
    zr_color_attachment_desc color;
    int32_t color_format;
    int32_t depth_format;
};

enum CmdType { C_BEGIN_RENDERING, C_END_RENDERING, C_BIND_PIPELINE, C_BIND_UNIFORM, C_SET_VIEWPORT, C_SET_SCISSOR,
               C_BIND_VB, C_BIND_IB, C_DRAW, C_SET_SHARD, C_CLEAR_IMAGE, C_SET_ROUTE_CAP, C_PUSH_CONSTANTS };

struct RenderingState {
    zr_rect2d area;
    bool has_color = false, has_depth = false;
    zr_rendering_attachment color{}, depth{};
};

struct Cmd {
    CmdType type;
    RenderingState rendering;
    const zr_pipeline* pipeline = nullptr;
    const zr_buffer* buffer = nullptr;
    uint64_t offset = 0, range = 0;
    uint32_t a = 0, b = 0, c = 0, d = 0;
    int32_t e = 0;
    zr_viewport vp{};
    zr_rect2d rect{};
    zr_exchange_fn exchange = nullptr;  // C_SET_SHARD with a partitioned setup
    void* exchange_user = nullptr;
};

struct zr_cmd_t {
    zr_device* dev;
    std::vector<Cmd> cmds;
    std::vector<uint8_t> push_data;  // C_PUSH_CONSTANTS payloads (Cmd::offset indexes it)
    zr_result err = ZR_SUCCESS;
    std::string err_msg;
    bool in_rendering = false;
    bool has_exchange = false;  // a partitioned shard: its collective is called per submit, never captured
    // Replay of an unchanged command list: its launches captured once into a HIP
    // graph (valid while the device's scratch generation is unchanged).
    hipGraphExec_t graph = nullptr;
    uint64_t graph_gen = 0;
    uint32_t eager_runs = 0;
    void drop_graph() {
        if (graph) (void)hipGraphExecDestroy(graph);
        graph = nullptr;
    }
};

struct zr_fence_t {
    zr_device* dev;
    hipEvent_t ev;
    bool submitted = false;
};

struct ScratchSet {
    TriCompact* records = nullptr;
    uint64_t records_cap = 0;  // primitives
    TriRecord* records_big = nullptr;
    uint64_t records_big_cap = 0;
    float4* mesh_edges = nullptr;
    uint64_t mesh_edges_cap = 0;
    BBox* bboxes = nullptr;
    uint64_t bboxes_cap = 0;
    uint32_t* tile_counts = nullptr;
    uint64_t tiles_cap = 0;
    uint32_t* draw_info = nullptr;  // k_setup_bin -> k_tile (kInfoWords)
    uint64_t draw_info_cap = 0;
    uint32_t* counters = nullptr;
    uint64_t counters_cap = 0;
    uint32_t* bins = nullptr;
    uint64_t bins_cap = 0;
    uint2* runs = nullptr;           // pool run table: [ntiles * run_cap] (DrawParams::runs)
    uint64_t runs_cap = 0;
    uint32_t* run_counts = nullptr;  // [ntiles] (zero between draws: k_tile resets it)
    uint64_t run_counts_cap = 0;
    uint32_t* tile_order = nullptr;  // k_tile's block -> tile schedule (k_setup_bin's last workgroup writes it)
    uint32_t* job_slot = nullptr;    // tile jobs (DrawParams::job_entries): key slot per split tile
    uint64_t job_slot_cap = 0;
    unsigned long long* job_keys = nullptr;  // [slots][kTilePixels] per-job key buffers
    uint64_t job_keys_cap = 0;
    uint32_t* job_tickets = nullptr;  // [slots], zero between draws
    uint64_t job_tickets_cap = 0;
    uint64_t tile_order_cap = 0;
    uint8_t* xsend = nullptr;   // partitioned setup: exchange blocks (bytes)
    uint64_t xsend_cap = 0;
    uint8_t* xrecv = nullptr;
    uint64_t xrecv_cap = 0;
    uint32_t* gids = nullptr;   // draw primitive per received position (records mode)
    uint64_t gids_cap = 0;
    uint64_t xsend_layout = 0;  // (shard count, route capacity) the send headers were last zeroed for
    hipEvent_t setup_done = nullptr;  // k_setup_bin of the last draw that used this set
    hipEvent_t route_done = nullptr;  // partitioned draws: k_route + exchange of the last draw that used this set
    hipEvent_t tile_done = nullptr;   // k_tile of the last draw that used this set
    bool tile_done_valid = false;
    // a draw on the main stream alone used this set after tile_done was recorded:
    // the event is recorded on the main stream only when a setup-stream draw next
    // needs this set (an event record between two frames costs ~4.4 us of idle GPU)
    bool main_reader_pending = false;
};

struct TimedLaunch {
    const char* name;
    hipEvent_t start, stop;
};

struct zr_device_t {
    int hip_device = 0;
    hipStream_t stream = nullptr;
    // Scratch (grow-only) in two sets: consecutive draws alternate, so the setup of
    // draw i+1 (on setup_stream) only waits for the tile pass of draw i-1, the last
    // reader of its set, and runs while the tile pass of draw i finishes.
    ScratchSet sets[kScratchSets];
    uint32_t cur_set = 0;
    hipStream_t setup_stream = nullptr;
    // partitioned draws: k_route + the exchange on a stream of their own, so draw
    // i+2's route and exchange, draw i+1's records-mode binning (setup_stream) and
    // draw i's tile pass (main stream) run together: a three-stage pipeline over
    // three scratch sets
    hipStream_t route_stream = nullptr;
    // k_setup_bin on the setup stream (two scratch sets), so draw i+1's setup
    // fills CUs draw i's tile pass frees.  Measured with round 1's two-launch
    // split setup (1 GPU): C1 (100k tris) 1180 -> 1274 Mtri/s, C2 7925 -> 8007,
    // C3 equal, C4 (10M) 25.1 -> 23.8 G (the co-running passes contend), so by
    // default only draws of <= 2^18 primitives overlapped, and tile-row shards (whose
    // tile pass leaves most CUs idle: C2 G=2/4/8 +2.8/+2.3/+0.7 %, C3 G=8 +7 %).
    // Re-measured with round 6's kernels (one setup workgroup per CU, slab
    // binning, spread allocators; docs/EXPERIMENTS.md round 6): C2 107.7 -> 95.5 us per frame, C3
    // 206.8 -> 196.9, c2x 155.2 -> 133.7, c3x 243.1 -> 216.5, but C4 316.9 -> 405.8
    // (its HBM-bound setup is the frame).  So draws of fewer primitives than
    // pixels overlap too (use_overlap_setup); ZR_SETUP_OVERLAP=0 / 1 forces it off / on.
    int setup_overlap = -1;
    int rec_table = -1;        // ZR_REC_TABLE=0/1 forces k_tile's record table (A/B); -1: use_record_table
    int tile_sched = -1;       // ZR_TILE_SCHED=0/1 forces the heaviest-first tile schedule (A/B); -1: use_tile_schedule
    uint32_t rec_wgs = 0;      // ZR_REC_WGS: k_setup_bin workgroups of partitioned (records-mode) draws; 0: one per CU
    int bin_stage = -1;        // ZR_BIN_STAGE: k_setup_bin phase 4 staged through LDS (1), direct (0), default (-1)
    int micro = -1;            // ZR_MICRO=0/1: setup's micro-primitive test off / on; -1: use_micro_test
    int cu_count = 0;
    uint32_t occupancy_checked_tiles = 0;
    bool occupancy_checked_mesh = false;
    uint32_t tile_threads = 0; // k_tile workgroup size override (ZR_TILE_NT: 256, 512; 0 = by tile count)
    uint32_t debug = 0;
    uint64_t initial_bins = 0;  // ZR_BIN_CAPACITY; 0 = bin_default_capacity of the first draw
    uint64_t bins_want = 0;     // bin buffer the last sync's draws asked for (+10 %; 0: none measured yet)
    uint64_t bins_want_max = 0; // ... the most any sync asked for since the last shrink check
    uint32_t bins_syncs = 0;    // syncs with draws since the last shrink check
    uint32_t shrink_syncs = kBinShrinkSyncs;  // ZR_BIN_SHRINK_SYNCS (0: never shrink)
    // slab targets (bin_slab_target) measured per draw shape, (tiles << 32) | primitives;
    // the draws since the last sync, in status-slot order (DrawParams::stat_slot)
    struct BinShape {
        uint32_t target = 0;    // bin_slab_target
        uint32_t pool = 0;      // pool entries its runs asked for (at the slab it had)
        uint32_t max_tile = 0;  // its longest tile list
        uint32_t job_bufs = 0;  // tile-job key buffers its split tiles needed (0: none built)
        uint32_t job_parts = 0; // ... and the most parts it put on one XCD
    };
    int jobs = -1;              // ZR_JOBS: tile jobs of N entries (tests), 0 off; -1: use_tile_jobs
    uint64_t job_want_max = 0;  // the most job keys (buffers x tile pixels) a draw asked for since the last shrink check
    std::vector<uint32_t> slab_tile_px;  // pixels per tile of the draw in each status slot (slab_keys)
    uint32_t setup_batch = 0;            // ZR_SETUP_BATCH: primitives per lane in flight (1, 2, 4; 0: 2)
    uint32_t forced_tile_shift = 0;      // ZR_TILE: every unsharded draw with a built instance at this edge (16 / 32 / 64)
    uint32_t last_tile = kTile;          // the tile edge of the last draw recorded
    std::unordered_map<uint64_t, BinShape> bin_shapes;
    std::vector<uint64_t> slab_keys;
    uint32_t forced_slab = ~0u; // ZR_BIN_SLAB: every draw's slab (tests: pool runs everywhere)
    unsigned long long* dbg_ts = nullptr;  // kDebugStamps
    uint32_t dbg_wgs = 0, dbg_tiles = 0;
    std::string dbg_ts_path;
    uint32_t* status_host = nullptr;
    uint32_t* status_dev = nullptr;
    // command lists submitted since the last sync point (in flight) + stats
    std::vector<zr_cmd*> pending;
    uint64_t overflowed_draws = 0;
    uint64_t route_fallbacks = 0;  // partitioned draws set up in full after a block overflow
    hipStream_t own_stream = nullptr;  // `stream` unless zr_device_set_stream installed the caller's
    // multi-GPU (zr_device_init_rccl): one communicator for the partitioned-setup
    // exchange (setup stream), one for the tile-row gather (gather stream), so an
    // exchange never queues behind the previous frame's gather
    void* comm_x = nullptr;
    void* comm_g = nullptr;
    int comm_rank = 0, comm_size = 1;
    hipStream_t gather_stream = nullptr;
    hipEvent_t frame_done = nullptr;
    uint8_t* gather_stage = nullptr;  // packed leftover-row rectangles of the row gather
    uint64_t gather_stage_cap = 0;
    zr_draw_stats last{};
    uint64_t last_prims = 0;
    // profiling (zr_device_set_profiling): 1 = per-kernel events, 2 = also the winner census
    bool profiling = false;
    int32_t census = 0;
    uint32_t* win_bits = nullptr;   // census bitmap of the last census draw (one bit per draw primitive)
    uint64_t win_bits_cap = 0;      // words
    uint64_t census_words = 0;      // words of the last census draw, read at the next sync point
    bool use_graphs = false;    // ZR_GRAPH=1: replay resubmitted command lists as HIP graphs
    bool capturing = false;     // inside hipStreamBeginCapture: no allocation allowed
    uint64_t scratch_gen = 0;   // bumped whenever a scratch buffer is reallocated
    std::vector<TimedLaunch> timed;
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, std::pair<double, uint64_t>> times;
};

// ------------------------------------------------------------ device helpers

namespace {

// A draw shape's key for the bin / job measurements (zr_device_t::bin_shapes):
// its tile count and its primitive count to 5 significant bits, so draws whose
// count varies a little (culling, LOD, streaming) share their measurements.
uint64_t shape_key(uint32_t ntiles, uint32_t prims) {
    const uint32_t bits = prims ? 32u - (uint32_t)__builtin_clz(prims) : 0u;
    const uint32_t drop = bits > 5u ? bits - 5u : 0u;
    return ((uint64_t)ntiles << 32) | ((prims >> drop) << drop);
}

zr_result set_device(zr_device* d) {
    ZR_HIP(hipSetDevice(d->hip_device));
    return ZR_SUCCESS;
}

hipEvent_t take_event(zr_device* d) {
    if (!d->event_pool.empty()) {
        hipEvent_t e = d->event_pool.back();
        d->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void collect_timings(zr_device* d) {
    for (auto& t : d->timed) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, t.start, t.stop) == hipSuccess) {
            auto& slot = d->times[t.name];
            slot.first += ms;
            slot.second += 1;
        }
        d->event_pool.push_back(t.start);
        d->event_pool.push_back(t.stop);
    }
    d->timed.clear();
}

template <typename F>
void timed_launch(zr_device* d, const char* name, hipStream_t stream, F&& fn) {
    if (!d->profiling) {
        fn();
        return;
    }
    TimedLaunch t{name, take_event(d), take_event(d)};
    (void)hipEventRecord(t.start, stream);
    fn();
    (void)hipEventRecord(t.stop, stream);
    d->timed.push_back(t);
}

// Both streams idle (scratch may be freed, host-visible status is final).
zr_result sync_streams(zr_device* d) {
    ZR_HIP(hipStreamSynchronize(d->route_stream));
    ZR_HIP(hipStreamSynchronize(d->setup_stream));
    ZR_HIP(hipStreamSynchronize(d->stream));
    if (d->gather_stream) ZR_HIP(hipStreamSynchronize(d->gather_stream));
    return ZR_SUCCESS;
}

template <typename T>
zr_result grow(zr_device* d, T*& ptr, uint64_t& cap, uint64_t need, uint64_t elem_bytes) {
    if (need <= cap && ptr) return ZR_SUCCESS;
    if (d->capturing) return ZR_NOT_READY;  // graph capture aborted: the caller runs eagerly
    d->scratch_gen++;
    zr_result rc = sync_streams(d);
    if (rc) return rc;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    uint64_t n = std::max<uint64_t>(need, 1024);
    void* p = nullptr;
    ZR_HIP(hipMalloc(&p, n * elem_bytes));
    ptr = (T*)p;
    cap = n;
    return ZR_SUCCESS;
}

zr_result execute(zr_device* d, zr_cmd* cmd);

// Events that only order this device's streams around data this device's own
// kernels write and read (setup_done, tile_done), never waited on by the host:
// device-scope release, no system-scope cache writeback when they are recorded.
// (Host waits go through hipStreamSynchronize or a fence's own event.)  The row
// gather's events keep the system-scope fence: RCCL moves the rows between devices.
#ifndef ZR_EVENT_SYSTEM_FENCE
constexpr unsigned kStreamEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;
#else
constexpr unsigned kStreamEventFlags = hipEventDisableTiming;
#endif

// kDebugStamps: per-phase durations of k_setup_bin across workgroups (us, 100 MHz clock).
void dump_stamps(zr_device* d) {
    std::vector<unsigned long long> ts(d->dbg_wgs * 8);
    if (hipMemcpy(ts.data(), d->dbg_ts, ts.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    FILE* f = fopen(d->dbg_ts_path.c_str(), "a");
    if (!f) return;
    unsigned long long t0 = ~0ull;
    for (uint32_t w = 0; w < d->dbg_wgs; ++w) t0 = std::min(t0, ts[w * 8]);
    fprintf(f, "wgs=%u", d->dbg_wgs);
    for (int i = 0; i <= 6; ++i) {
        double mn = 1e30, mx = 0, sum = 0;
        for (uint32_t w = 0; w < d->dbg_wgs; ++w) {
            const double v = (double)(ts[w * 8 + i] - t0) * 0.01;
            mn = std::min(mn, v); mx = std::max(mx, v); sum += v;
        }
        fprintf(f, " s%d[min %.1f avg %.1f max %.1f]", i, mn, sum / d->dbg_wgs, mx);
    }
    // phase-1 duration per workgroup, by blockIdx % 8 (a label for workgroups that share an XCD)
    double xs[8] = {0}, xn[8] = {0};
    fprintf(f, "\n  p1 by w%%8:");
    for (uint32_t w = 0; w < d->dbg_wgs; ++w) {
        xs[w % 8] += (double)(ts[w * 8 + 1] - ts[w * 8]) * 0.01;
        xn[w % 8] += 1;
    }
    for (int x = 0; x < 8; ++x) fprintf(f, " %.1f", xn[x] ? xs[x] / xn[x] : 0.0);
    {
        std::vector<unsigned long long> tt(d->dbg_tiles * 8);
        if (d->dbg_tiles && hipMemcpy(tt.data(), d->dbg_ts + 8192 * 8, tt.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            unsigned long long t1 = ~0ull;
            for (uint32_t w = 0; w < d->dbg_tiles; ++w) t1 = std::min(t1, tt[w * 8]);
            fprintf(f, "\n  tile(us from first tile start; dur = per-tile phase length):");
            // t0 start, t1 init, t2 first segment sorted, t3 raster done, t5 resolve
            // winners known, t6 first batch fetched, t4 resolve done
            for (int i : {0, 1, 2, 3, 5, 6, 4}) {
                double mn = 1e30, mx = 0, sum = 0, dsum = 0, dmx = 0;
                for (uint32_t w = 0; w < d->dbg_tiles; ++w) {
                    const double v = (double)(tt[w * 8 + i] - t1) * 0.01;
                    mn = std::min(mn, v); mx = std::max(mx, v); sum += v;
                    const int prev = i == 5 ? 3 : i == 6 ? 5 : i == 4 ? 6 : i - 1;
                    if (i) { const double dd = (double)(tt[w * 8 + i] - tt[w * 8 + prev]) * 0.01; dsum += dd; dmx = std::max(dmx, dd); }
                }
                fprintf(f, " t%d[min %.1f avg %.1f max %.1f dur avg %.1f max %.1f]", i, mn, sum / d->dbg_tiles, mx,
                        dsum / d->dbg_tiles, dmx);
            }
        }
    }
    {  // raw per-tile stamps for offline analysis: <path>.tiles.csv
        std::vector<unsigned long long> tt(d->dbg_tiles * 8);
        if (d->dbg_tiles && hipMemcpy(tt.data(), d->dbg_ts + 8192 * 8, tt.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            FILE* g = fopen((d->dbg_ts_path + ".tiles.csv").c_str(), "a");
            if (g) {
                unsigned long long t1 = ~0ull;
                for (uint32_t w = 0; w < d->dbg_tiles; ++w) t1 = std::min(t1, tt[w * 8]);
                fprintf(g, "tile,t0,t1,t2,t3,t4,t5,nbig,count,lane_steps,wave_sweeps\n");
                for (uint32_t w = 0; w < d->dbg_tiles; ++w) {
                    fprintf(g, "%u", w);
                    for (int i = 0; i <= 4; ++i) fprintf(g, ",%.2f", (double)(tt[w * 8 + i] - t1) * 0.01);
                    // 512-thread tiles: t5 = the first segment's chunks done, nbig = its
                    // wave-path queue (256: resolve_tile's own stamps, in t5 / the count word)
                    fprintf(g, ",%.2f,%llu,%llu,%llu,%llu\n", (double)(tt[w * 8 + 5] - t1) * 0.01, tt[w * 8 + 6] >> 32,
                            tt[w * 8 + 6] & 0xFFFFFFFFull, tt[w * 8 + 7] & 0xFFFFFFFFull, tt[w * 8 + 7] >> 32);
                }
                fclose(g);
            }
        }
    }
    fprintf(f, "\n  p1 first 16 wgs:");
    for (uint32_t w = 0; w < std::min(16u, d->dbg_wgs); ++w) fprintf(f, " %.1f", (double)(ts[w * 8 + 1] - ts[w * 8]) * 0.01);
    fprintf(f, "\n  p1 last 16 wgs:");
    for (uint32_t w = d->dbg_wgs > 16 ? d->dbg_wgs - 16 : 0; w < d->dbg_wgs; ++w)
        fprintf(f, " %.1f", (double)(ts[w * 8 + 1] - ts[w * 8]) * 0.01);
    fprintf(f, "\n");
    fclose(f);
}

zr_result device_sync(zr_device* d) {
    zr_result rc = set_device(d);
    if (rc) return rc;
    if ((rc = sync_streams(d))) return rc;
    collect_timings(d);
    volatile uint32_t* st = d->status_host;
    d->last.bin_pairs = st[kStTotalPairs];
    d->last.triangles_setup = st[kStTrianglesSetup];
    d->last.triangles_dropped_clip = st[kStDroppedClip];
    d->last.micro_fragments = st[kStMicro];
    d->last.bin_pool_pairs = st[kStPoolPairs];
    d->last.bin_pool_runs = st[kStPoolRuns];
    d->last.tile_jobs = st[kStJobs];
    st[kStJobsDenied] = 0;  // (a denied split is sized from its shape's kStJobBufSlot0 below)
    // partitioned draws since the previous sync point
    if (st[kStRouteMax]) {  // kept from the last interval with partitioned draws
        d->last.route_max_entries = st[kStRouteMax];
        st[kStRouteMax] = 0;
    }
    d->route_fallbacks += st[kStRouteFallback];
    d->last.route_fallback_draws = d->route_fallbacks;
    st[kStRouteFallback] = 0;
    d->pending.clear();
    if (d->dbg_ts && !d->dbg_ts_path.empty()) dump_stamps(d);
    // Bin buffer sizing: later draws take slabs of the target the
    // draws since the last sync asked for, and the buffer grows to what they asked
    // for -- slabs plus the pool their runs needed -- when it is smaller (a draw with
    // a dropped run rasterized that tile by k_tile's record scan).  Every
    // kBinShrinkSyncs syncs it shrinks to the most any of them asked for when it is
    // more than twice that and the difference is worth it (kBinShrinkMin): not
    // per sync (a device alternating between a light and a heavy scene would
    // reallocate, and drop runs, every time), and not for a few MB (a shrink of
    // the 8-way shard emulation's small buffers cost one rank 7 us per frame).  (Capped at 2^30
    // entries, 4 GiB: a larger draw keeps using the exact spill path.)
    uint64_t need = st[kStBinNeed];  // (draws with a dropped run; the others from their slots)
    st[kStBinNeed] = 0;
    for (size_t i = 0; i < d->slab_keys.size(); ++i) {
        const uint32_t target = st[kStSlabSlot0 + i], pool = st[kStPoolSlot0 + i], max_tile = st[kStMaxSlot0 + i];
        const uint32_t job_bufs = st[kStJobBufSlot0 + i], job_parts = st[kStJobPartSlot0 + i];
        st[kStJobBufSlot0 + i] = 0;
        st[kStJobPartSlot0 + i] = 0;
        d->job_want_max = std::max<uint64_t>(d->job_want_max, (uint64_t)job_bufs * d->slab_tile_px[i]);
        if (!target) continue;
        need = std::max<uint64_t>({need, (d->slab_keys[i] >> 32) * target + pool,
                                   (d->slab_keys[i] >> 32) * bin_slab_whole(target, max_tile) + 4096});
        st[kStSlabSlot0 + i] = 0;
        st[kStPoolSlot0 + i] = 0;
        st[kStMaxSlot0 + i] = 0;
        if (d->bin_shapes.size() >= 1024) d->bin_shapes.clear();  // (shapes that come and go)
        zr_device_t::BinShape& v = d->bin_shapes[d->slab_keys[i]];
        if (v.target != target || v.pool != pool) d->scratch_gen++;  // recorded graphs bake the slab in
        if (use_tile_jobs(v.max_tile) != use_tile_jobs(max_tile)) d->scratch_gen++;
        if (v.job_bufs != job_bufs || v.job_parts != job_parts) d->scratch_gen++;
        v.target = target;
        v.pool = pool;
        v.max_tile = max_tile;
        v.job_bufs = job_bufs;
        v.job_parts = job_parts;
    }
    d->slab_keys.clear();
    d->slab_tile_px.clear();
    if (st[kStOverflow]) {
        d->overflowed_draws += st[kStOverflow];
        st[kStOverflow] = 0;
    }
    if (need) {
        d->bins_want = std::min<uint64_t>(std::max<uint64_t>(need + need / 10 + 4096, 1ull << 20), 1ull << 30);
        d->bins_want_max = std::max(d->bins_want_max, d->bins_want);
        const bool check = d->shrink_syncs && ++d->bins_syncs >= d->shrink_syncs;
        for (ScratchSet& S : d->sets) {
            const bool shrink = check && S.bins_cap > 2 * d->bins_want_max && S.bins_cap - d->bins_want_max >= kBinShrinkMin;
            if (!S.bins || (S.bins_cap >= need && !shrink)) continue;
            ZR_HIP(hipFree(S.bins));
            S.bins = nullptr;
            void* p = nullptr;
            const uint64_t size = check ? d->bins_want_max : d->bins_want;
            ZR_HIP(hipMalloc(&p, size * 4));
            S.bins = (uint32_t*)p;
            S.bins_cap = size;
            d->scratch_gen++;
        }
        if (check) {
            // tile-job key buffers (8 B per pixel of a tile each) follow the most
            // any draw of the interval asked for, the same way
            const uint64_t keep = d->job_want_max ? d->job_want_max * 5 / 4 + 16 * (uint64_t)kTilePixels : 0;  // (keys)
            for (ScratchSet& S : d->sets) {
                if (!S.job_keys || S.job_keys_cap <= 2 * keep + (1u << 16)) continue;
                (void)hipFree(S.job_keys);
                (void)hipFree(S.job_tickets);
                S.job_keys = nullptr;
                S.job_tickets = nullptr;
                S.job_keys_cap = S.job_tickets_cap = 0;
                d->scratch_gen++;
            }
            d->job_want_max = 0;
            d->bins_want_max = 0;
            d->bins_syncs = 0;
        }
    }
    d->last.tile_size = d->last_tile;
    d->last.job_key_bytes = 0;
    for (const ScratchSet& S : d->sets) d->last.job_key_bytes += S.job_keys ? S.job_keys_cap * 8 : 0;
    d->last.overflowed_draws = d->overflowed_draws;
    d->last.bin_capacity = d->sets[0].bins_cap;
    for (const ScratchSet& S : d->sets)
        if (S.bins) d->last.bin_capacity = std::min<uint64_t>(d->last.bin_capacity, S.bins_cap);
    if (d->census_words) {  // distinct primitives that won a pixel in the last census draw
        std::vector<uint32_t> bits(d->census_words);
        ZR_HIP(hipMemcpy(bits.data(), d->win_bits, bits.size() * 4, hipMemcpyDeviceToHost));
        uint64_t n = 0;
        for (uint32_t w : bits) n += (uint64_t)__builtin_popcount(w);
        d->last.winners = n;
        d->census_words = 0;
    }
    return ZR_SUCCESS;
}

// ------------------------------------------------------------ draw execution

struct VertexBinding {
    const zr_buffer* buf = nullptr;
    uint64_t offset = 0;
};

struct ExecState {
    const zr_pipeline* pipe = nullptr;
    bool vp_set = false, sc_set = false;
    zr_viewport vp{};
    zr_rect2d sc{};
    VertexBinding vb[8];
    const zr_buffer* ib = nullptr;
    uint64_t ib_offset = 0;
    int32_t index_type = 0;
    std::map<std::pair<uint32_t, uint32_t>, std::pair<const zr_buffer*, uint64_t>> ubos;
    bool rendering = false;
    RenderingState rs;
    bool color_clear_pending = false, depth_clear_pending = false;
    uint32_t shard_rank = 0, shard_count = 1;
    zr_exchange_fn exchange = nullptr;
    void* exchange_user = nullptr;
    uint32_t route_cap = 0;  // entries per exchange block (zr_cmd_set_route_capacity; 0: route_capacity_default)
    // push-constant state (vkCmdPushConstants): bytes, which 4-byte words were
    // written, and the layout they were written with
    float push[kMaxPushWords] = {};
    uint32_t push_written = 0;
    const zr_pipeline* push_layout = nullptr;
};

// Entries per exchange block when the caller sets none: every primitive of the
// range for two ranks or fewer, else twice a uniform share plus a margin.  A block
// that still overflows is exact (its receiver sets up the whole draw), only slower.
uint64_t route_capacity_default(uint64_t span, uint64_t G) {
    if (G <= 2) return span;
    return std::min<uint64_t>(span, (2 * span + G - 1) / G + 4096);
}

int32_t choose_depth_mode(bool test, bool write, int32_t op) {
    if (!test) return kDepthLastWins;
    if (write) {
        switch (op) {
        case 1: return kDepthMinStrict;
        case 3: return kDepthMinNonStrict;
        case 4: return kDepthMaxStrict;
        case 6: return kDepthMaxNonStrict;
        default: break;
        }
    }
    return kDepthLastWins;
}

// The draw's tiles at an edge of 1 << shift pixels: the grid, and the tiles this
// shard owns (ShardGeom).
void set_tiles(DrawParams& P, uint32_t shift) {
    const uint32_t t = 1u << shift;
    P.tile_shift = shift;
    P.tiles_x = (P.fb_w + t - 1) >> shift;
    P.tiles_y = (P.fb_h + t - 1) >> shift;
    const ShardGeom sg = shard_geom(P.tiles_x, P.tiles_y, P.shard_count, P.shard_rank);
    P.full_rows = sg.full_rows;
    P.own_rows = sg.own_rows;
    P.left_lo = sg.left_lo;
    P.left_hi = sg.left_hi;
    P.ntiles = shard_tiles(sg);
}

zr_result fill_target(const ExecState& s, DrawParams& P) {
    const zr_texture* ct = s.rs.has_color ? s.rs.color.texture : nullptr;
    const zr_texture* dt = s.rs.has_depth ? s.rs.depth.texture : nullptr;
    if (!ct && !dt) return fail(ZR_ERROR_VALIDATION_FAILED, "render pass without attachments");
    const zr_texture* ref = ct ? ct : dt;
    if (ct && dt && (ct->width != dt->width || ct->height != dt->height))
        return fail(ZR_ERROR_VALIDATION_FAILED, "colour and depth attachment extents differ");
    if (dt && dt->format != ZR_FORMAT_D32_SFLOAT) return fail(ZR_ERROR_FORMAT_NOT_SUPPORTED, "depth format");
    if (ct && format_bpp(ct->format) == 0) return fail(ZR_ERROR_FORMAT_NOT_SUPPORTED, "colour format");
    P.fb_w = ref->width;
    P.fb_h = ref->height;
    P.color = ct ? (uint8_t*)ct->ptr : nullptr;
    P.color_format = ct ? ct->format : 0;
    P.color_bpp = ct ? ct->bpp : 0;
    P.depth = dt ? (float*)dt->ptr : nullptr;
    const int32_t ax0 = std::max(0, s.rs.area.x), ay0 = std::max(0, s.rs.area.y);
    const int64_t ax1 = std::min<int64_t>((int64_t)s.rs.area.x + s.rs.area.width, P.fb_w) - 1;
    const int64_t ay1 = std::min<int64_t>((int64_t)s.rs.area.y + s.rs.area.height, P.fb_h) - 1;
    P.ra_x0 = ax0;
    P.ra_y0 = ay0;
    P.ra_x1 = (int32_t)ax1;
    P.ra_y1 = (int32_t)ay1;
    P.shard_rank = s.shard_rank;
    P.shard_count = s.shard_count;
    set_tiles(P, kTileShift);
    // clears (fused into the first draw of the pass, else k_clear at end_rendering)
    P.clear_color_enable = (ct && s.color_clear_pending) ? 1u : 0u;
    if (ct) {
        for (int i = 0; i < 4; ++i) P.clear_color[i] = s.rs.color.clear_value[i];
        P.clear_color_packed = pack_rgba8(P.clear_color, ct->format, kSrgbThresholds);
    }
    P.clear_depth_enable = (dt && s.depth_clear_pending) ? 1u : 0u;
    P.clear_depth = dt ? s.rs.depth.clear_value[0] : 1.0f;
    P.load_depth = (dt && !s.depth_clear_pending) ? 1u : 0u;
    return ZR_SUCCESS;
}

zr_result ensure_scratch(zr_device* d, ScratchSet& S, DrawParams& P) {
    zr_result rc;
    // the mesh program's fans 1 and 2 have records and bboxes of their own
    const uint64_t prims = std::max<uint64_t>(P.prims, 1) * (P.program == kProgMesh ? kMeshFans : 1u);
    if ((rc = grow(d, S.records, S.records_cap, prims, sizeof(TriCompact)))) return rc;
    if ((rc = grow(d, S.records_big, S.records_big_cap, prims, sizeof(TriRecord)))) return rc;
    if ((rc = grow(d, S.bboxes, S.bboxes_cap, prims, sizeof(BBox)))) return rc;
    if (P.program == kProgMesh && (rc = grow(d, S.mesh_edges, S.mesh_edges_cap, std::max<uint64_t>(P.prims, 1) * 3u,
                                             sizeof(float4))))
        return rc;
    {  // per-tile counters start at zero; k_setup_bin leaves them zero after every draw
        const uint64_t cap = S.tiles_cap;
        if ((rc = grow(d, S.tile_counts, S.tiles_cap, P.ntiles + 1, 4))) return rc;
        if (S.tiles_cap != cap) ZR_HIP(hipMemset(S.tile_counts, 0, S.tiles_cap * 4));
    }
    if ((rc = grow(d, S.draw_info, S.draw_info_cap, kInfoWords, 4))) return rc;
    if (!S.counters) {  // zeroed once; k_setup_bin leaves them zero after every draw
        if ((rc = grow(d, S.counters, S.counters_cap, kCtWords, 4))) return rc;
        ZR_HIP(hipMemset(S.counters, 0, S.counters_cap * 4));
    }
    {  // per-tile run words start at zero; k_tile leaves them zero after every draw
        const uint64_t cap = S.run_counts_cap;
        if ((rc = grow(d, S.run_counts, S.run_counts_cap, P.ntiles + 1, 4))) return rc;
        if (S.run_counts_cap != cap) ZR_HIP(hipMemset(S.run_counts, 0, S.run_counts_cap * 4));
    }
    P.run_cap = std::min<uint32_t>(P.setup_wgs, kMaxRunsPerTile);
    {  // run tables start empty (length 0); k_tile clears the ones it used
        const uint64_t cap = S.runs_cap;
        if ((rc = grow(d, S.runs, S.runs_cap, (uint64_t)P.ntiles * P.run_cap, sizeof(uint2)))) return rc;
        if (S.runs_cap != cap) ZR_HIP(hipMemset(S.runs, 0, S.runs_cap * sizeof(uint2)));
    }
    if (!S.bins) {
        const uint64_t want = std::max(d->bins_want, d->initial_bins ? d->initial_bins : bin_default_capacity(prims, P.ntiles));
        if ((rc = grow(d, S.bins, S.bins_cap, want, 4))) return rc;
    }
    if (!S.setup_done) {
        ZR_HIP(hipEventCreateWithFlags(&S.setup_done, kStreamEventFlags));
        ZR_HIP(hipEventCreateWithFlags(&S.tile_done, kStreamEventFlags));
        ZR_HIP(hipEventCreateWithFlags(&S.route_done, kStreamEventFlags));
    }
    P.records = S.records;
    P.records_big = S.records_big;
    P.mesh_edges = S.mesh_edges;
    P.bboxes = S.bboxes;
    P.tile_counts = S.tile_counts;
    P.draw_info = S.draw_info;
    P.counters = S.counters;
    P.bins = S.bins;
    P.runs = S.runs;
    P.run_counts = S.run_counts;
    // tile t's slab is bins[t * slab, (t + 1) * slab), the pool the rest.  Before
    // any measurement of the draw's shape: slabs of a third of the buffer.  After:
    // the buffer less the pool the shape's runs asked for (+25 %, and at least a
    // 64th of the buffer) over the tiles, but no less than the shape's target --
    // a buffer larger than the pairs need (the 2^20-entry floor; C2's 2 x prims)
    // goes to the slabs, where no run is needed (cerberus: the target slab put its
    // crowded tiles' excess in runs, setup +8 us).
    const uint64_t nt = std::max<uint32_t>(P.ntiles, 1u), cap = S.bins_cap;
    const uint64_t key = shape_key(P.ntiles, P.draw_prims);
    const auto shape = d->bin_shapes.find(key);
    uint64_t slab = cap / (3 * nt);
    if (d->forced_slab != ~0u) {
        slab = d->forced_slab;
    } else if (shape != d->bin_shapes.end()) {
        const uint64_t pool = std::max<uint64_t>((uint64_t)shape->second.pool * 5 / 4 + 4096, cap / 64);
        slab = std::max<uint64_t>({shape->second.target, bin_slab_whole(shape->second.target, shape->second.max_tile),
                                   cap > pool ? (cap - pool) / nt : 0});
    }
    slab = std::min<uint64_t>({slab, cap / nt, (uint64_t)kMaxSlab});
    P.slab = (uint32_t)slab;
    P.pool_off = (uint32_t)(slab * P.ntiles);
    P.pool_cap = (uint32_t)(S.bins_cap - slab * P.ntiles);
    // Tile jobs (DrawParams::job_entries): for a shape whose longest list was long
    // (use_tile_jobs), or forced (ZR_JOBS).  The grid's spare blocks bound the jobs
    // beyond one per tile by the shape's pairs / J (pairs < tiles x target).
    P.job_entries = 0;
    P.job_pad = P.job_slots = 0;
    const bool known = shape != d->bin_shapes.end();
    if (!(d->debug & kDebugPhase1Only)) {
        // (a shape not measured yet may be skewed: its first draw builds jobs for
        // whatever lists turn out long -- the clustered c2x scene's first frame
        // walked its 30-segment tile in one workgroup -- at the cost of the job
        // builder and the spare blocks once)
        if (d->jobs > 0)
            P.job_entries = (uint32_t)d->jobs;
        else if (d->jobs < 0 && (!known || use_tile_jobs(shape->second.max_tile)))
            P.job_entries = kTileJobEntries;
    }
    if (P.job_entries) {
        // Key buffers (one per job of a split tile, kTilePixels x 8 B each) and the
        // grid's spare part blocks (job_pad / 8 per XCD: a tile's parts go to its
        // XCD).  A shape whose split was measured gets what it needed (+25 %): a draw
        // that did not fit is counted and rasterized unsplit, and the next draw of
        // its shape is sized from what it asked for.  A shape not measured yet gets
        // what the bin buffer's pairs can need at most -- each part past the first
        // holds job_entries pairs, each split tile more than job_entries -- within a
        // fixed memory bound (kJobKeyBytesFirst).
        uint64_t bufs, parts;
        if (known && shape->second.job_bufs) {
            bufs = (uint64_t)shape->second.job_bufs * 5 / 4 + 16;
            parts = (uint64_t)shape->second.job_parts * 5 / 4 + 8;
        } else {
            const uint64_t pairs = known ? (uint64_t)P.ntiles * shape->second.target + shape->second.pool : cap;
            bufs = std::min<uint64_t>(2 * (pairs / P.job_entries) + 64, kJobKeyBytesFirst / (8ull << (2 * P.tile_shift)));
            parts = pairs / P.job_entries / 4 + 64;  // (a few crowded tiles: parts spread over several XCDs)
        }
        P.job_pad = (uint32_t)std::min<uint64_t>(8 * parts, 1u << 20);
        P.job_slots = (uint32_t)std::min<uint64_t>(bufs, 1u << 20);
        const uint64_t tc = S.job_tickets_cap;
        if ((rc = grow(d, S.job_slot, S.job_slot_cap, P.ntiles, 4))) return rc;
        if ((rc = grow(d, S.job_keys, S.job_keys_cap, (uint64_t)P.job_slots << (2 * P.tile_shift), 8))) return rc;
        if ((rc = grow(d, S.job_tickets, S.job_tickets_cap, P.job_slots, 4))) return rc;
        if (S.job_tickets_cap != tc) ZR_HIP(hipMemset(S.job_tickets, 0, S.job_tickets_cap * 4));
        P.job_slot = S.job_slot;
        P.job_keys = S.job_keys;
        P.job_tickets = S.job_tickets;
    }
    P.stat_slot = ~0u;
    if (!d->capturing && d->slab_keys.size() < kSlabSlots) {
        P.stat_slot = (uint32_t)d->slab_keys.size();
        d->slab_keys.push_back(key);
        d->slab_tile_px.push_back(1u << (2 * P.tile_shift));
    }
    P.status = d->status_dev;
    return ZR_SUCCESS;
}

zr_result rccl_exchange(void* user, void* stream, const void* send, void* recv, uint64_t bytes_per_rank);
zr_result replay_exchange(void* user, void* stream, const void* send, void* recv, uint64_t bytes_per_rank);

zr_result exec_draw(zr_device* d, ExecState& s, const Cmd& c, bool indexed) {
    if (!s.rendering) return fail(ZR_ERROR_VALIDATION_FAILED, "draw outside begin_rendering/end_rendering");
    // the runtime's own all-to-all sends one block to every communicator rank and
    // takes bit d of a route mask for comm rank d: the shard must be that communicator
    if (s.exchange == &rccl_exchange &&
        (s.exchange_user != (void*)d || !d->comm_x || d->comm_size != (int)s.shard_count ||
         d->comm_rank != (int)s.shard_rank))
        return fail(ZR_ERROR_VALIDATION_FAILED,
                    "tile shard (rank, count) differs from the device's RCCL communicator (zr_device_init_rccl)");
    const zr_pipeline* pp = s.pipe;
    if (!pp) return fail(ZR_ERROR_VALIDATION_FAILED, "draw without a bound pipeline");
    if (!s.vp_set || !s.sc_set)
        return fail(ZR_ERROR_VALIDATION_FAILED, "dynamic viewport/scissor not set (pipeline.rs:734)");
    if (pp->color_count != (s.rs.has_color ? 1u : 0u))
        return fail(ZR_ERROR_VALIDATION_FAILED, "node colour targets do not match pipeline colour attachments");
    if (!s.vb[0].buf) return fail(ZR_ERROR_VALIDATION_FAILED, "vertex buffer binding 0 not bound");
    if (indexed && !s.ib) return fail(ZR_ERROR_VALIDATION_FAILED, "draw_indexed without an index buffer");

    DrawParams P;
    memset(&P, 0, sizeof P);
    zr_result rc = fill_target(s, P);
    if (rc) return rc;
    // A tile-row shard that owns no row of this target draws nothing, but a
    // partitioned one still routes its range and joins the exchange (every rank
    // calls the collective once per draw, zenith_raster.h).
    const bool no_tiles = P.ntiles == 0;
    if (no_tiles && !s.exchange) return ZR_SUCCESS;
    if (!pp->has_fs) {
        P.color = nullptr;
        P.color_bpp = 0;
    }
    const uint64_t count = c.a, instances = c.b;
    const uint64_t tpi = count / 3u;
    const uint64_t prims = tpi * instances;
    if (prims > kBinPrimMask) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "more than 2^26-1 primitives in one draw");
    if (P.fb_w > 16384 || P.fb_h > 16384) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "attachment larger than 16384");

    const zr_buffer* vb = s.vb[0].buf;
    P.vb = (const uint8_t*)vb->ptr + s.vb[0].offset;
    P.vb_bytes = vb->size > s.vb[0].offset ? vb->size - s.vb[0].offset : 0;
    P.stride = pp->stride;
    P.nattr = pp->nattr;
    for (int i = 0; i < 4; ++i) {
        P.attr_offset[i] = pp->attr_offset[i];
        P.attr_size[i] = pp->attr_size[i];
    }
    {  // one compare per vertex in the kernels instead of one per (vertex, attribute)
        uint64_t end = 0;
        for (uint32_t a = 0; a < P.nattr; ++a) end = std::max<uint64_t>(end, (uint64_t)P.attr_offset[a] + P.attr_size[a]);
        P.vid_count = P.nattr == 0 ? (1ull << 32) : (P.vb_bytes < end ? 0ull : (P.vb_bytes - end) / P.stride + 1ull);
    }
    if (indexed) {
        P.ib = (const uint8_t*)s.ib->ptr + s.ib_offset;
        P.ib_bytes = s.ib->size > s.ib_offset ? s.ib->size - s.ib_offset : 0;
        P.index_size = s.index_type == ZR_INDEX_TYPE_UINT16 ? 2u : 4u;
        P.first = c.c;
        P.vertex_offset = c.e;
        const uint64_t nidx = P.ib_bytes / 4;  // only read for u32 indices (k_setup_bin fetch_indices_gid)
        P.ib_tris = nidx > P.first ? (uint32_t)std::min<uint64_t>((nidx - P.first) / 3, 0xFFFFFFFFull) : 0u;
    } else {
        P.ib_tris = 0;
        P.index_size = 0;
        P.first = c.c;
        P.vertex_offset = 0;
    }
    P.tris_per_instance = (uint32_t)tpi;
    P.prims = (uint32_t)prims;
    P.draw_prims = (uint32_t)prims;
    // Partitioned setup: this rank routes [lo, hi) of the draw's
    // primitives; the setup pass then runs over the received blocks' dense
    // positions (at most shard_count * span of them).
    const bool partitioned = s.exchange != nullptr;
    const bool mesh = pp->program == kProgMesh;
    if (partitioned && mesh)
        return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "partitioned tile shards do not route clipped (mesh program) draws");
    if (mesh && prims * kMeshFans > kBinPrimMask)
        return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "mesh program: more than (2^26-1)/3 primitives in one draw");
    uint64_t positions = prims;
    uint64_t span = 0;
    if (partitioned) {
        const uint64_t G = s.shard_count;
        const uint64_t per_rank = (prims + G - 1) / G;
        span = std::max<uint64_t>(1, (per_rank + kRouteChunk - 1) / kRouteChunk) * kRouteChunk;
        const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(span, s.route_cap ? s.route_cap : route_capacity_default(span, G)));
        // received entries, or every draw primitive when a block overflowed
        positions = std::max<uint64_t>(prims, G * cap);
        if (positions > kBinPrimMask)
            return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "partitioned draw: more than 2^26-1 block positions");
        P.route_cap = (uint32_t)cap;
        if (s.exchange == &replay_exchange) {
            // the recorded blocks are copied into this draw's receive buffer (G blocks)
            const zr_replay_exchange* r = (const zr_replay_exchange*)s.exchange_user;
            if (!r || !r->src || r->bytes != G * route_block_bytes(P.route_cap))
                return fail(ZR_ERROR_VALIDATION_FAILED,
                            "zr_replay_exchange_fn: recorded bytes differ from this draw's exchange layout "
                            "(shard count x route_block_bytes(route capacity))");
        }
        P.route_chunks = (uint32_t)(span / kRouteChunk);
        P.route_lo = (uint32_t)std::min<uint64_t>(prims, (uint64_t)s.shard_rank * span);
        P.route_hi = (uint32_t)std::min<uint64_t>(prims, (uint64_t)P.route_lo + span);
        P.prims = (uint32_t)positions;
    }
    // viewport transform constants (Vulkan 1.3 §Controlling the Viewport)
    P.hw = s.vp.width * 0.5f;
    P.hh = s.vp.height * 0.5f;
    P.cx = s.vp.x + P.hw;
    P.cy = s.vp.y + P.hh;
    P.dr = s.vp.max_depth - s.vp.min_depth;
    P.dmin = s.vp.min_depth;
    P.dlo = std::min(s.vp.min_depth, s.vp.max_depth);
    P.dhi = std::max(s.vp.min_depth, s.vp.max_depth);
    P.clip_x0 = std::max<int32_t>(s.sc.x, P.ra_x0);
    P.clip_y0 = std::max<int32_t>(s.sc.y, P.ra_y0);
    P.clip_x1 = (int32_t)std::min<int64_t>((int64_t)s.sc.x + s.sc.width - 1, P.ra_x1);
    P.clip_y1 = (int32_t)std::min<int64_t>((int64_t)s.sc.y + s.sc.height - 1, P.ra_y1);
    P.cull_mode = pp->cull_mode;
    P.front_face = pp->front_face;
    P.write_mask = pp->color.write_mask;
    // depth
    const bool has_depth = P.depth != nullptr;
    const bool test = has_depth && pp->has_depth_state && pp->ds.depth_test_enable;
    const bool write = test && pp->ds.depth_write_enable;
    const int32_t op = test ? pp->ds.depth_compare_op : 7;
    if (write && op == 5) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "NOT_EQUAL with depth writes");
    P.depth_mode = choose_depth_mode(test, write, op);
    P.depth_op = op;
    P.depth_write_out = write ? 1u : 0u;
    // shading
    P.program = pp->program;
    P.time_ptr = nullptr;
    for (const auto& b : pp->bindings) {
        auto it = s.ubos.find({b.set, b.binding});
        if (it == s.ubos.end())
            return fail(ZR_ERROR_VALIDATION_FAILED, std::string("descriptor '") + b.name + "' not bound");
        if (pp->program == kProgTriangle && !strcmp(b.name, "Time")) {
            if (it->second.second + 4 > it->second.first->size)
                return fail(ZR_ERROR_VALIDATION_FAILED, "Time uniform range out of bounds");
            P.time_ptr = (const float*)((const uint8_t*)it->second.first->ptr + it->second.second);
        }
        if (pp->program == kProgMesh && !strcmp(b.name, "View")) {
            if (it->second.second + 64 > it->second.first->size || (it->second.second & 3u))
                return fail(ZR_ERROR_VALIDATION_FAILED, "View uniform range out of bounds (float4x4 view_proj)");
            P.view_proj = (const float*)((const uint8_t*)it->second.first->ptr + it->second.second);
        }
    }
    if (pp->view_push) {
        // mesh_push.slang: View.view_proj is push-constant bytes [0, 64)
        if ((s.push_written & 0xFFFFu) != 0xFFFFu)
            return fail(ZR_ERROR_VALIDATION_FAILED, "push constants [0, 64) (View.view_proj) not pushed before the draw");
        if (s.push_layout != pp && (!s.push_layout || s.push_layout->push_ranges.size() != pp->push_ranges.size() ||
                                    !std::equal(pp->push_ranges.begin(), pp->push_ranges.end(),
                                                s.push_layout->push_ranges.begin(),
                                                [](const zr_push_constant_range& a, const zr_push_constant_range& b) {
                                                    return a.stage_flags == b.stage_flags && a.offset == b.offset &&
                                                           a.size == b.size;
                                                })))
            return fail(ZR_ERROR_VALIDATION_FAILED,
                        "push constants were pushed with a layout whose ranges differ from the bound pipeline's");
        memcpy(P.push, s.push, sizeof P.push);
        P.view_push = 1;
        P.view_proj = nullptr;
    }
    if (mesh && !P.view_proj && !P.view_push) return fail(ZR_ERROR_VALIDATION_FAILED, "descriptor 'View' not bound");
    // The tile edge (tile_shift_for): 16 px for a shape whose 32-px tiles needed
    // tile jobs (measured), 64 px for large dense targets, 32 px otherwise and for
    // shards; ZR_TILE forces an edge (tests, A/B) where the instance exists.
    if (P.shard_count == 1 && tile_variant_built(P.program, P.depth_mode)) {
        uint32_t shift = d->forced_tile_shift;
        if (!shift) {
            // the edge by size, then 16 px if that edge's shape was measured crowded
            // (its draws keep consulting that measurement, stable once it is made)
            shift = tile_shift_for(prims, P.fb_w, P.fb_h, P.shard_count, false);
            if (shift != P.tile_shift) set_tiles(P, shift);
            const auto sh = d->bin_shapes.find(shape_key(P.ntiles, P.draw_prims));
            if (sh != d->bin_shapes.end() && crowded_shape(sh->second.max_tile, sh->second.target))
                shift = tile_shift_for(prims, P.fb_w, P.fb_h, P.shard_count, true);
        }
        if (shift != P.tile_shift) set_tiles(P, shift);
        if (P.ntiles > kMaxTilesPerPass) set_tiles(P, kTileShift);
    }
    d->last_tile = 1u << P.tile_shift;
    // binning geometry: k_setup_bin runs one kSetupThreads workgroup per CU at most
    // (its LDS histogram of all tiles; workgroups never wait for each other)
    if (P.ntiles > kMaxTilesPerPass)
        return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "more owned tiles in one pass than the setup pass histogram holds (kMaxTilesPerPass)");
    P.setup_batch = mesh ? 1u : (d->setup_batch ? d->setup_batch : 2u);  // k_setup_bin<2> (the mesh instance: <1, true>)
    const uint64_t lds_budget = kSetupLdsBudget;  // (one workgroup per CU owns the LDS; two measured slower)
    if (d->occupancy_checked_tiles != P.ntiles || d->occupancy_checked_mesh != mesh) {
        int nb = 0;
        ZR_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, setup_bin_kernel(P.setup_batch, mesh), kSetupThreads,
                                                            setup_bin_lds_bytes(P.ntiles, 0)));
        if (nb < 1) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "k_setup_bin cannot be resident on a CU");
        d->occupancy_checked_tiles = P.ntiles;
        d->occupancy_checked_mesh = mesh;
    }
    uint64_t stage_entries = 0;
    {
        // one workgroup per CU (fewer for small draws); a wave processes units of
        // 64 * batch * 2^k primitives, at most ~64 units per workgroup on average
        // (at most kMaxRunsPerTile workgroups: a pool run takes its workgroup's slot
        // of the tile's run table)
        const uint64_t cus = std::min<uint64_t>((uint64_t)std::max(d->cu_count, 1), kMaxRunsPerTile);
        const uint64_t per_wg = (uint64_t)kSetupThreads * P.setup_batch;
        P.setup_wgs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(cus, (positions + per_wg - 1) / per_wg));
        if (partitioned)  // records mode: sized to the expected received entries (ZR_REC_WGS: A/B)
            P.setup_wgs = std::min<uint32_t>(P.setup_wgs, d->rec_wgs ? d->rec_wgs
                                                                     : records_setup_wgs((uint64_t)s.shard_count * P.route_cap,
                                                                                         (uint32_t)cus));
        uint32_t shift = 6;
        while ((1u << shift) < 64u * P.setup_batch) ++shift;
        while (((positions + (1ull << shift) - 1) >> shift) > 64ull * P.setup_wgs) ++shift;
        P.unit_shift = shift;
        P.units = (uint32_t)std::max<uint64_t>(1, (positions + (1ull << shift) - 1) >> shift);
        // a workgroup's bboxes live in LDS when they fit beside the histograms
        const uint64_t own_max = ((uint64_t)P.units + P.setup_wgs - 1) / P.setup_wgs;
        const uint64_t entries = own_max << shift;
        const uint64_t hist = setup_bin_lds_bytes(P.ntiles, 0);
        const uint64_t budget = std::min<uint64_t>(kSetupBboxLdsBytes, hist < lds_budget ? lds_budget - hist : 0);
        // (mesh: fans 1 and 2 keep their bboxes in global memory, so all of them do)
        P.bbox_lds = (!mesh && entries * sizeof(BBox) <= budget) ? (uint32_t)entries : 0u;
        stage_entries = entries;
    }
    // k_setup_bin on the setup stream with two scratch sets (zr_device_t::setup_overlap);
    // not while debugging or with graph replay, whose captures bake in set 0
    const bool overlap_setup = (d->setup_overlap > 0 || (d->setup_overlap < 0 && use_overlap_setup(prims, P.fb_w, P.fb_h, P.shard_count))) &&
                       !d->use_graphs && !d->debug;
    // k_setup_bin phase 4 staged in LDS (pairs grouped by tile, stored run by run):
    // room for twice the workgroup's primitives, in the CU's LDS that setup owns
    // alone -- not beside a tile pass (overlapped setup), whose workgroups would
    // lose the LDS (C1 frame +1.9 us).  A workgroup whose pairs do not fit
    // scatters straight to the bins.
    {
        const uint64_t used = setup_bin_lds_bytes(P.ntiles, P.bbox_lds);
        const uint64_t cur = ((uint64_t)P.ntiles + 3u) / 4u * 4u * 4u;
        const uint64_t room = used + cur < lds_budget ? (lds_budget - used - cur) / 8u : 0u;
        const uint64_t cap = std::min<uint64_t>(room, 2u * std::max<uint64_t>(stage_entries, 1024u));
        const bool on = d->bin_stage > 0 || (d->bin_stage < 0 && kBinStageDefault && !overlap_setup);
        P.bin_stage = on && cap >= 1024u ? (uint32_t)cap : 0u;
    }
    // (records mode never runs setup_finish: no effect there)
    P.micro = (d->micro < 0 ? use_micro_test(prims, (uint64_t)(P.ra_x1 - P.ra_x0 + 1) * (uint64_t)(P.ra_y1 - P.ra_y0 + 1))
                            : d->micro != 0) ? 1u : 0u;
    P.tile_threads = (d->tile_threads && P.tile_shift == kTileShift)
                         ? d->tile_threads
                         : tile_threads_for(P.ntiles, (uint32_t)std::max(d->cu_count, 1), prims, partitioned, P.tile_shift);
    P.rec_table = (d->rec_table < 0 ? use_record_table(prims, P.tiles_x, P.tiles_y, P.tile_shift) : d->rec_table != 0) ? 1u : 0u;
    const bool sched = d->tile_sched < 0 ? use_tile_schedule(P.ntiles, (uint32_t)std::max(d->cu_count, 1), P.tile_threads,
                                                             prims, P.tile_shift)
                                         : d->tile_sched != 0;
    P.debug = d->debug;
    if (d->census && !d->capturing) {  // winner census: a bitmap over the draw's primitives, zeroed per draw
        const uint64_t words = ((uint64_t)P.draw_prims + 31u) / 32u + 1u;
        if ((rc = grow(d, d->win_bits, d->win_bits_cap, words, 4))) return rc;
        ZR_HIP(hipMemsetAsync(d->win_bits, 0, words * 4, d->stream));
        P.win_bits = d->win_bits;
        d->census_words = words;
    }
    if (d->debug & kDebugStamps) {
        if (!d->dbg_ts) ZR_HIP(hipMalloc((void**)&d->dbg_ts, (8192 + kMaxTilesPerPass) * 8 * sizeof(unsigned long long)));
        P.dbg_ts = d->dbg_ts;
        d->dbg_wgs = P.setup_wgs;
        d->dbg_tiles = P.ntiles;
    }
    // Overlapped and partitioned draws alternate between the two scratch sets.
    // Partitioned draws always do: the route, exchange and setup of draw i+1 run
    // on setup_stream while draw i's tile pass runs on the main stream.
    // (ZR_SETUP_OVERLAP=0 serialises partitioned draws too: a diagnostic that times
    // each of their kernels alone)
    const bool overlap = (partitioned && d->setup_overlap != 0) || overlap_setup;
    ScratchSet& S = d->sets[overlap ? d->cur_set : 0];
    if (overlap) d->cur_set = (d->cur_set + 1u) % kScratchSets;
    if ((rc = ensure_scratch(d, S, P))) return rc;
    // (a phase-1-only timing run never reaches the last workgroup's ticket, so it
    // writes no schedule: k_tile then keeps xcd_tile order instead of reading an
    // unwritten one)
    P.tile_sched = sched && !(d->debug & kDebugPhase1Only) ? 1u : 0u;
    if ((sched || P.job_entries) && !(d->debug & kDebugPhase1Only)) {
        if ((rc = grow(d, S.tile_order, S.tile_order_cap, (uint64_t)P.ntiles + P.job_pad, 4))) return rc;
        P.tile_order = S.tile_order;
    }
    d->last_prims = prims;
    d->last.triangles_in = prims;

    const hipStream_t ss = overlap ? d->setup_stream : d->stream;
    // partitioned: route + exchange on their own stream (serialised: the device stream)
    const hipStream_t rs = overlap ? d->route_stream : d->stream;
    // the first pass into this scratch set may start once its previous reader (the
    // k_tile kScratchSets draws back) is done
    if (overlap && S.main_reader_pending) {
        // everything enqueued on the main stream so far includes that last reader
        ZR_HIP(hipEventRecord(S.tile_done, d->stream));
        S.tile_done_valid = true;
        S.main_reader_pending = false;
    }
    if (overlap && S.tile_done_valid) ZR_HIP(hipStreamWaitEvent(partitioned ? rs : ss, S.tile_done, 0));
    // debug early exits skip the self-reset at the end of k_setup_bin; the memsets
    // go on the stream that runs this draw's k_setup_bin, so they precede it
    // (partitioned: after the route, which waited for the set's last reader)
    auto debug_resets = [&]() -> zr_result {
        if (d->debug) {
            ZR_HIP(hipMemsetAsync(P.counters, 0, kCtWords * 4, ss));
            ZR_HIP(hipMemsetAsync(P.tile_counts, 0, (size_t)P.ntiles * 4, ss));
            ZR_HIP(hipMemsetAsync(P.run_counts, 0, (size_t)P.ntiles * 4, ss));
        }
        return ZR_SUCCESS;
    };
    if (!partitioned && (rc = debug_resets())) return rc;
    if (partitioned) {
        const uint64_t bytes = (uint64_t)s.shard_count * route_block_bytes(P.route_cap);
        if ((rc = grow(d, S.xsend, S.xsend_cap, bytes, 1))) return rc;
        if ((rc = grow(d, S.xrecv, S.xrecv_cap, bytes, 1))) return rc;
        if ((rc = grow(d, S.gids, S.gids_cap, positions, 4))) return rc;
        // The send headers' totals are k_route's counters: zero when the block
        // layout is new; afterwards this rank's records-mode setup re-zeroes them
        // once the exchange has consumed them (a rank without rows: below).
        const uint64_t block = route_block_bytes(P.route_cap);
        const uint64_t layout = ((uint64_t)s.shard_count << 32) | P.route_cap;
        auto zero_headers = [&]() -> zr_result {
            ZR_HIP(hipMemset2DAsync(S.xsend, block, 0, sizeof(RouteHeader), s.shard_count, rs));
            return ZR_SUCCESS;
        };
        if (S.xsend_layout != layout) {
            if ((rc = zero_headers())) return rc;
            S.xsend_layout = layout;
        }
        P.route_out = S.xsend;
        P.gids = S.gids;
        timed_launch(d, "route", rs, [&] { launch_route(P, rs); });
        ZR_HIP(hipGetLastError());
        zr_result xr = ZR_SUCCESS;
        timed_launch(d, "exchange", rs, [&] {
            xr = s.exchange(s.exchange_user, (void*)rs, S.xsend, S.xrecv, route_block_bytes(P.route_cap));
        });
        if (xr != ZR_SUCCESS) {
            // the route's totals stay in the send headers (no records-mode setup will
            // consume and re-zero them): the next draw on this set memsets them first
            S.xsend_layout = 0;
            return fail(xr, "tile-shard exchange callback failed: " + g_last_error);
        }
        P.rlist = S.xrecv;
        if (no_tiles) {  // routed and exchanged; nothing of this target to draw here
            if ((rc = zero_headers())) return rc;  // (no records-mode setup to reset them)
            // joined back into the device stream like every other setup-stream pass, so
            // a fence (or a caller stream waiting on the device stream) covers the
            // route's reads of the caller's vertex and index buffers
            ZR_HIP(hipEventRecord(S.route_done, rs));
            ZR_HIP(hipStreamWaitEvent(d->stream, S.route_done, 0));
            s.color_clear_pending = false;
            s.depth_clear_pending = false;
            return ZR_SUCCESS;
        }
        if (rs != ss) {  // the binning stage waits for this draw's exchange
            ZR_HIP(hipEventRecord(S.route_done, rs));
            ZR_HIP(hipStreamWaitEvent(ss, S.route_done, 0));
        }
        if ((rc = debug_resets())) return rc;
        // Records-mode setup (binning the received records) runs on the setup
        // stream behind the exchange, so draw i+1's route, exchange and binning
        // overlap draw i's tile pass (the main stream only runs tile passes;
        // DESIGN.md §7).  k_setup_bin has no grid barrier, so sharing the GPU with
        // the collectives' kernels is safe.
        timed_launch(d, "setup_bin", ss, [&] { launch_setup_bin(P, ss); });
        ZR_HIP(hipEventRecord(S.setup_done, ss));
        ZR_HIP(hipStreamWaitEvent(d->stream, S.setup_done, 0));
    } else {
        timed_launch(d, "setup_bin", ss, [&] { launch_setup_bin(P, ss); });
        if (overlap) {
            ZR_HIP(hipEventRecord(S.setup_done, ss));
            ZR_HIP(hipStreamWaitEvent(d->stream, S.setup_done, 0));
        }
    }
    timed_launch(d, "tile", d->stream, [&] { launch_tile(P, d->stream); });
    // Every draw marks its set's last reader: a later draw that sets up on
    // setup_stream into this set waits for it.  An overlapped draw records its own
    // tile_done right here (the next setup into the other set must not wait for
    // it); a draw on the main stream alone only flags the set, and the event is
    // recorded when an overlapped draw next needs the set (above), so back-to-back
    // single-stream frames carry no event at all.
    // (A graph capture uses set 0 only; submit_graph_or_eager flags it after the replay.)
    if (!d->capturing) {
        if (overlap) {
            ZR_HIP(hipEventRecord(S.tile_done, d->stream));
            S.tile_done_valid = true;
            S.main_reader_pending = false;
        } else {
            S.main_reader_pending = true;
        }
    }
    ZR_HIP(hipGetLastError());
    s.color_clear_pending = false;
    s.depth_clear_pending = false;
    return ZR_SUCCESS;
}

zr_result exec_end_rendering(zr_device* d, ExecState& s) {
    if (s.color_clear_pending || s.depth_clear_pending) {
        DrawParams P;
        memset(&P, 0, sizeof P);
        zr_result rc = fill_target(s, P);
        if (rc) return rc;
        timed_launch(d, "clear", d->stream, [&] { launch_clear(P, d->stream); });
        ZR_HIP(hipGetLastError());
    }
    s.rendering = false;
    s.color_clear_pending = s.depth_clear_pending = false;
    return ZR_SUCCESS;
}

zr_result execute(zr_device* d, zr_cmd* cmd) {
    ExecState s;
    for (const Cmd& c : cmd->cmds) {
        zr_result rc = ZR_SUCCESS;
        switch (c.type) {
        case C_BEGIN_RENDERING:
            s.rendering = true;
            s.rs = c.rendering;
            for (const zr_texture* t : {s.rs.has_color ? s.rs.color.texture : nullptr,
                                        s.rs.has_depth ? s.rs.depth.texture : nullptr}) {
                if (!t || !t->gather_pending) continue;
                if (d->capturing) return ZR_NOT_READY;  // a gather is not part of the graph: run eagerly
                ZR_HIP(hipStreamWaitEvent(d->stream, t->gather_done, 0));
            }
            s.color_clear_pending = s.rs.has_color && s.rs.color.load_op == ZR_ATTACHMENT_LOAD_OP_CLEAR;
            s.depth_clear_pending = s.rs.has_depth && s.rs.depth.load_op == ZR_ATTACHMENT_LOAD_OP_CLEAR;
            break;
        case C_END_RENDERING: rc = exec_end_rendering(d, s); break;
        case C_CLEAR_IMAGE: {
            // the k_clear of a render pass with LOAD_OP_CLEAR and no draw, over the
            // whole image on every rank (not a tile-row shard)
            if (s.rendering) { rc = fail(ZR_ERROR_VALIDATION_FAILED, "clear_color_image inside a render pass"); break; }
            ExecState cs;
            cs.rendering = true;
            cs.rs = c.rendering;
            cs.color_clear_pending = true;
            const zr_texture* t = c.rendering.color.texture;
            if (t->gather_pending) {
                if (d->capturing) return ZR_NOT_READY;
                ZR_HIP(hipStreamWaitEvent(d->stream, t->gather_done, 0));
            }
            rc = exec_end_rendering(d, cs);
            break;
        }
        case C_BIND_PIPELINE: s.pipe = c.pipeline; break;
        case C_BIND_UNIFORM: s.ubos[{c.a, c.b}] = {c.buffer, c.offset}; break;
        case C_SET_VIEWPORT: s.vp = c.vp; s.vp_set = true; break;
        case C_SET_SCISSOR: s.sc = c.rect; s.sc_set = true; break;
        case C_BIND_VB:
            if (c.a < 8) s.vb[c.a] = {c.buffer, c.offset};
            break;
        case C_BIND_IB: s.ib = c.buffer; s.ib_offset = c.offset; s.index_type = c.e; break;
        case C_DRAW: rc = exec_draw(d, s, c, c.d != 0); break;
        case C_SET_SHARD:
            s.shard_rank = c.a;
            s.shard_count = c.b;
            s.exchange = c.exchange;
            s.exchange_user = c.exchange_user;
            break;
        case C_SET_ROUTE_CAP: s.route_cap = c.a; break;
        case C_PUSH_CONSTANTS:
            memcpy((uint8_t*)s.push + c.a, cmd->push_data.data() + c.offset, c.b);
            for (uint32_t w = c.a / 4u; w < (c.a + c.b) / 4u; ++w) s.push_written |= 1u << w;
            s.push_layout = c.pipeline;
            break;
        }
        if (rc) return rc;
    }
    if (s.rendering) return exec_end_rendering(d, s);
    return ZR_SUCCESS;
}

void latch(zr_cmd* cmd, zr_result rc, const std::string& msg) {
    if (cmd->err == ZR_SUCCESS) {
        cmd->err = rc;
        cmd->err_msg = msg;
    }
}

}  // namespace

// ======================================================================= ABI

extern "C" {

ZR_API const char* zr_last_error_message(void) { return g_last_error.c_str(); }

ZR_API const char* zr_build_info(void) {
    return "libzenith_raster (HIP, gfx950): setup/scan/bin/tile passes, tile=32x32, 64-bit LDS visibility keys";
}

ZR_API zr_result zr_device_create(int32_t hip_device, zr_device** out) {
    if (!out) return fail(ZR_ERROR_VALIDATION_FAILED, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(ZR_ERROR_INITIALIZATION_FAILED, "no HIP device available");
    if (hip_device < 0 || hip_device >= n) return fail(ZR_ERROR_INITIALIZATION_FAILED, "bad device index");
    zr_device* d = new (std::nothrow) zr_device_t();
    if (!d) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "device alloc");
    d->hip_device = hip_device;
    if (const char* dbg = getenv("ZR_DEBUG")) d->debug = (uint32_t)strtoul(dbg, nullptr, 0);
    if (const char* p = getenv("ZR_DEBUG_TS")) d->dbg_ts_path = p;
    // (at most 2^30 entries: k_setup_bin's cursors tag pending and dropped runs in bits 30-31)
    if (const char* cap = getenv("ZR_BIN_CAPACITY"))
        d->initial_bins = std::min<uint64_t>(std::max<uint64_t>(64, strtoull(cap, nullptr, 0)), 1ull << 30);
    if (const char* sl = getenv("ZR_BIN_SLAB")) d->forced_slab = (uint32_t)std::min<uint64_t>(strtoull(sl, nullptr, 0), kMaxSlab);
    if (const char* g = getenv("ZR_GRAPH")) d->use_graphs = strtoul(g, nullptr, 0) != 0;
    if (const char* o = getenv("ZR_SETUP_OVERLAP")) d->setup_overlap = strtoul(o, nullptr, 0) != 0 ? 1 : 0;
    if (const char* rt = getenv("ZR_REC_TABLE")) d->rec_table = strtoul(rt, nullptr, 0) != 0 ? 1 : 0;
    if (const char* ts = getenv("ZR_TILE_SCHED")) d->tile_sched = strtoul(ts, nullptr, 0) != 0 ? 1 : 0;
    if (const char* rw = getenv("ZR_REC_WGS")) d->rec_wgs = (uint32_t)strtoul(rw, nullptr, 0);
    if (const char* bs = getenv("ZR_BIN_STAGE")) d->bin_stage = atoi(bs);
    if (const char* mi = getenv("ZR_MICRO")) d->micro = atoi(mi) != 0 ? 1 : 0;
    if (const char* ss = getenv("ZR_BIN_SHRINK_SYNCS")) d->shrink_syncs = (uint32_t)strtoul(ss, nullptr, 0);
    if (const char* jb = getenv("ZR_JOBS")) d->jobs = atoi(jb) > 0 ? std::max(atoi(jb), 256) : 0;
    if (const char* sb = getenv("ZR_SETUP_BATCH")) {
        const int b = atoi(sb);
        d->setup_batch = b == 1 || b == 2 || b == 4 ? (uint32_t)b : 0u;
    }
    if (const char* tl = getenv("ZR_TILE")) {
        const unsigned long v = strtoul(tl, nullptr, 0);
        d->forced_tile_shift = v == 16 ? 4u : v == 32 ? 5u : v == 64 ? 6u : 0u;
    }
    if (const char* nt = getenv("ZR_TILE_NT")) {
        const unsigned long v = strtoul(nt, nullptr, 0);
        d->tile_threads = v >= 512 ? 512u : v ? 256u : 0u;
    }
    ZR_HIP(hipSetDevice(hip_device));
    ZR_HIP(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    d->own_stream = d->stream;
    ZR_HIP(hipStreamCreateWithFlags(&d->setup_stream, hipStreamNonBlocking));
    ZR_HIP(hipStreamCreateWithFlags(&d->route_stream, hipStreamNonBlocking));
    for (uint32_t b : {1u, 2u, 4u})  // histograms + bbox array may exceed the 64 KB default
        ZR_HIP(hipFuncSetAttribute(setup_bin_kernel(b, false), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)kSetupLdsBudget));
    ZR_HIP(hipFuncSetAttribute(setup_bin_kernel(1, true), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)kSetupLdsBudget));
    ZR_HIP(hipDeviceGetAttribute(&d->cu_count, hipDeviceAttributeMultiprocessorCount, hip_device));
    void* st = nullptr;
    ZR_HIP(hipHostMalloc(&st, kStWords * 4, hipHostMallocMapped));
    memset(st, 0, kStWords * 4);
    d->status_host = (uint32_t*)st;
    void* sd = nullptr;
    ZR_HIP(hipHostGetDevicePointer(&sd, st, 0));
    d->status_dev = (uint32_t*)sd;
    *out = d;
    return ZR_SUCCESS;
}

ZR_API void zr_device_destroy(zr_device* d) {
    if (!d) return;
    (void)hipSetDevice(d->hip_device);
    (void)hipStreamSynchronize(d->route_stream);
    (void)hipStreamSynchronize(d->setup_stream);
    (void)hipStreamSynchronize(d->stream);
    collect_timings(d);
    for (hipEvent_t e : d->event_pool) (void)hipEventDestroy(e);
    if (d->dbg_ts) (void)hipFree(d->dbg_ts);
    if (d->win_bits) (void)hipFree(d->win_bits);
    for (ScratchSet& S : d->sets) {
        for (void* p : {(void*)S.job_slot, (void*)S.job_keys, (void*)S.job_tickets, (void*)S.runs, (void*)S.run_counts, (void*)S.records, (void*)S.records_big, (void*)S.mesh_edges, (void*)S.bboxes, (void*)S.tile_counts,
                        (void*)S.draw_info, (void*)S.counters, (void*)S.bins, (void*)S.xsend, (void*)S.xrecv,
                        (void*)S.gids, (void*)S.tile_order})
            if (p) (void)hipFree(p);
        if (S.setup_done) (void)hipEventDestroy(S.setup_done);
        if (S.route_done) (void)hipEventDestroy(S.route_done);
        if (S.tile_done) (void)hipEventDestroy(S.tile_done);
    }
    (void)hipHostFree(d->status_host);
    rccl_comm_destroy(d->comm_x);
    rccl_comm_destroy(d->comm_g);
    if (d->gather_stream) (void)hipStreamDestroy(d->gather_stream);
    if (d->gather_stage) (void)hipFree(d->gather_stage);
    if (d->frame_done) (void)hipEventDestroy(d->frame_done);
    (void)hipStreamDestroy(d->setup_stream);
    (void)hipStreamDestroy(d->route_stream);
    (void)hipStreamDestroy(d->own_stream);
    delete d;
}

ZR_API zr_result zr_device_set_stream(zr_device* d, void* hip_stream) {
    if (!d) return fail(ZR_ERROR_VALIDATION_FAILED, "device is NULL");
    zr_result rc = device_sync(d);
    if (rc) return rc;
    d->stream = hip_stream ? (hipStream_t)hip_stream : d->own_stream;
    return ZR_SUCCESS;
}

ZR_API void* zr_device_stream(const zr_device* d) { return d ? (void*)d->stream : nullptr; }

ZR_API zr_result zr_device_wait_idle(zr_device* d) {
    if (!d) return fail(ZR_ERROR_VALIDATION_FAILED, "device is NULL");
    return device_sync(d);
}

ZR_API zr_result zr_device_set_profiling(zr_device* d, int32_t enable) {
    if (!d) return fail(ZR_ERROR_VALIDATION_FAILED, "device is NULL");
    d->profiling = enable != 0;
    d->census = enable >= 2 ? 1 : 0;
    return ZR_SUCCESS;
}

ZR_API int32_t zr_device_kernel_times(zr_device* d, zr_kernel_time* out, int32_t capacity, int32_t reset) {
    if (!d) return 0;
    int32_t n = 0;
    for (const auto& kv : d->times) {
        if (out && n < capacity) {
            memset(&out[n], 0, sizeof(zr_kernel_time));
            snprintf(out[n].name, sizeof(out[n].name), "%s", kv.first.c_str());
            out[n].total_ms = kv.second.first;
            out[n].launches = kv.second.second;
        }
        ++n;
    }
    if (reset) d->times.clear();
    return std::min(n, capacity);
}

ZR_API zr_result zr_device_last_draw_stats(zr_device* d, zr_draw_stats* out) {
    if (!d || !out) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    *out = d->last;
    return ZR_SUCCESS;
}

// ------------------------------------------------------------------ buffers

static zr_result buffer_make(zr_device* d, const zr_buffer_desc* desc, void* ext, zr_buffer** out) {
    if (!d || !desc || !out) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    *out = nullptr;
    zr_result rc = set_device(d);
    if (rc) return rc;
    zr_buffer* b = new (std::nothrow) zr_buffer_t();
    if (!b) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "buffer alloc");
    b->dev = d;
    b->size = desc->size;
    b->name = desc->name ? desc->name : "";
    b->external = ext != nullptr;
    if (ext) {
        b->ptr = ext;
    } else {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, std::max<uint64_t>(desc->size, 16));
        if (e != hipSuccess) {
            delete b;
            return fail(ZR_ERROR_OUT_OF_DEVICE_MEMORY, "hipMalloc failed for buffer " + std::string(desc->name ? desc->name : ""));
        }
        b->ptr = p;
    }
    *out = b;
    return ZR_SUCCESS;
}

ZR_API zr_result zr_buffer_create(zr_device* d, const zr_buffer_desc* desc, zr_buffer** out) {
    return buffer_make(d, desc, nullptr, out);
}

ZR_API zr_result zr_buffer_create_external(zr_device* d, const zr_buffer_desc* desc, void* ptr, zr_buffer** out) {
    if (!ptr) return fail(ZR_ERROR_VALIDATION_FAILED, "external pointer is NULL");
    return buffer_make(d, desc, ptr, out);
}

ZR_API void zr_buffer_destroy(zr_buffer* b) {
    if (!b) return;
    device_sync(b->dev);
    if (!b->external) (void)hipFree(b->ptr);
    delete b;
}

ZR_API zr_result zr_buffer_write(zr_buffer* b, uint64_t offset, const void* src, uint64_t size) {
    if (!b) return fail(ZR_ERROR_VALIDATION_FAILED, "buffer is NULL");
    if (size == 0) return ZR_SUCCESS;  // buffer.rs:301-303
    if (offset > b->size || size > b->size - offset)
        return fail(ZR_ERROR_OUT_OF_DEVICE_MEMORY, "write past the end of buffer '" + b->name + "'");
    zr_result rc = device_sync(b->dev);
    if (rc) return rc;
    ZR_HIP(hipMemcpyAsync((uint8_t*)b->ptr + offset, src, size, hipMemcpyHostToDevice, b->dev->stream));
    ZR_HIP(hipStreamSynchronize(b->dev->stream));
    return ZR_SUCCESS;
}

ZR_API zr_result zr_buffer_read(zr_buffer* b, uint64_t offset, void* dst, uint64_t size) {
    if (!b) return fail(ZR_ERROR_VALIDATION_FAILED, "buffer is NULL");
    if (offset > b->size || size > b->size - offset) return fail(ZR_ERROR_VALIDATION_FAILED, "read out of range");
    zr_result rc = device_sync(b->dev);
    if (rc) return rc;
    ZR_HIP(hipMemcpyAsync(dst, (const uint8_t*)b->ptr + offset, size, hipMemcpyDeviceToHost, b->dev->stream));
    ZR_HIP(hipStreamSynchronize(b->dev->stream));
    return ZR_SUCCESS;
}

ZR_API uint64_t zr_buffer_size(const zr_buffer* b) { return b ? b->size : 0; }
ZR_API void* zr_buffer_device_address(const zr_buffer* b) { return b ? b->ptr : nullptr; }

// ----------------------------------------------------------------- textures

static zr_result texture_make(zr_device* d, const zr_texture_desc* desc, void* ext, zr_texture** out) {
    if (!d || !desc || !out) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    *out = nullptr;
    uint32_t bpp = desc->format == ZR_FORMAT_D32_SFLOAT ? 4u : format_bpp(desc->format);
    if (!bpp) return fail(ZR_ERROR_FORMAT_NOT_SUPPORTED, "unsupported texture format");
    if (desc->width == 0 || desc->height == 0) return fail(ZR_ERROR_VALIDATION_FAILED, "zero extent");
    zr_result rc = set_device(d);
    if (rc) return rc;
    zr_texture* t = new (std::nothrow) zr_texture_t();
    if (!t) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "texture alloc");
    t->dev = d;
    t->width = desc->width;
    t->height = desc->height;
    t->format = desc->format;
    t->bpp = bpp;
    t->external = ext != nullptr;
    t->name = desc->name ? desc->name : "";
    if (ext) {
        t->ptr = ext;
    } else {
        void* p = nullptr;
        if (hipMalloc(&p, (size_t)desc->width * desc->height * bpp) != hipSuccess) {
            delete t;
            return fail(ZR_ERROR_OUT_OF_DEVICE_MEMORY, "hipMalloc failed for texture");
        }
        t->ptr = p;
    }
    *out = t;
    return ZR_SUCCESS;
}

ZR_API zr_result zr_texture_create(zr_device* d, const zr_texture_desc* desc, zr_texture** out) {
    return texture_make(d, desc, nullptr, out);
}

ZR_API zr_result zr_texture_create_external(zr_device* d, const zr_texture_desc* desc, void* ptr, zr_texture** out) {
    if (!ptr) return fail(ZR_ERROR_VALIDATION_FAILED, "external pointer is NULL");
    return texture_make(d, desc, ptr, out);
}

ZR_API void zr_texture_destroy(zr_texture* t) {
    if (!t) return;
    device_sync(t->dev);
    if (!t->external) (void)hipFree(t->ptr);
    if (t->gather_done) (void)hipEventDestroy(t->gather_done);
    delete t;
}

ZR_API zr_result zr_texture_read(zr_texture* t, void* dst, uint64_t size) {
    if (!t || !dst) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    const uint64_t bytes = (uint64_t)t->width * t->height * t->bpp;
    if (size < bytes) return fail(ZR_ERROR_VALIDATION_FAILED, "destination too small");
    zr_result rc = device_sync(t->dev);
    if (rc) return rc;
    ZR_HIP(hipMemcpyAsync(dst, t->ptr, bytes, hipMemcpyDeviceToHost, t->dev->stream));
    ZR_HIP(hipStreamSynchronize(t->dev->stream));
    return ZR_SUCCESS;
}

ZR_API zr_result zr_texture_write(zr_texture* t, const void* src, uint64_t size) {
    if (!t || !src) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    const uint64_t bytes = (uint64_t)t->width * t->height * t->bpp;
    if (size < bytes) return fail(ZR_ERROR_VALIDATION_FAILED, "source too small");
    zr_result rc = device_sync(t->dev);
    if (rc) return rc;
    ZR_HIP(hipMemcpyAsync(t->ptr, src, bytes, hipMemcpyHostToDevice, t->dev->stream));
    ZR_HIP(hipStreamSynchronize(t->dev->stream));
    return ZR_SUCCESS;
}

ZR_API void* zr_texture_device_address(const zr_texture* t) { return t ? t->ptr : nullptr; }

// ------------------------------------------------------------------ shaders

ZR_API zr_result zr_shader_lookup(zr_device* d, const char* path, const char* entry, uint32_t stage, zr_shader** out) {
    (void)d;
    if (!out || !path || !entry) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    *out = nullptr;
    const std::string base = basename_of(path);
    for (const auto& s : kShaders) {
        if (base == s.file && !strcmp(entry, s.entry) && stage == s.stage) {
            zr_shader* sh = new (std::nothrow) zr_shader_t();
            if (!sh) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "shader alloc");
            sh->program = s.program;
            sh->stage = s.stage;
            sh->file = s.file;
            sh->entry = s.entry;
            sh->bindings.assign(s.bind, s.bind + s.nbind);
            sh->inputs.assign(s.inputs, s.inputs + s.ninputs);
            sh->push_constant_size = s.push_size;
            *out = sh;
            return ZR_SUCCESS;
        }
    }
    return fail(ZR_ERROR_SHADER_NOT_FOUND, "no built-in stage for " + base + ":" + entry);
}

ZR_API void zr_shader_destroy(zr_shader* sh) { delete sh; }

ZR_API int32_t zr_shader_bindings(const zr_shader* sh, zr_shader_binding* out, int32_t capacity) {
    if (!sh) return 0;
    const int32_t n = (int32_t)sh->bindings.size();
    for (int32_t i = 0; out && i < std::min(n, capacity); ++i) out[i] = sh->bindings[i];
    return n;
}

ZR_API uint32_t zr_shader_push_constant_size(const zr_shader* sh) { return sh ? sh->push_constant_size : 0u; }

ZR_API int32_t zr_shader_vertex_inputs(const zr_shader* sh, zr_vertex_input_attr* out, int32_t capacity) {
    if (!sh) return 0;
    const int32_t n = (int32_t)sh->inputs.size();
    for (int32_t i = 0; out && i < std::min(n, capacity); ++i) out[i] = sh->inputs[i];
    return n;
}

// ---------------------------------------------------------------- pipelines

// validate_vertex_inputs, zenith-rhi/src/pipeline.rs:228-287 (strict match).
static zr_result validate_vertex_inputs(const zr_shader* vs, const zr_vertex_attribute* attrs, uint32_t n,
                                        zr_pipeline_error* err) {
    if (vs->inputs.empty()) {
        if (n == 0) return ZR_SUCCESS;
        return fail(ZR_ERROR_VERTEX_INPUT_REFLECTION_MISSING,
                    "vertex shader reflection contains no vertex_inputs, but vertex_attributes were provided");
    }
    std::map<uint32_t, int32_t> expected, provided;
    for (const auto& vi : vs->inputs) expected[vi.location] = vi.format;
    for (uint32_t i = 0; i < n; ++i) {
        auto it = provided.find(attrs[i].location);
        if (it != provided.end()) {
            if (it->second != attrs[i].format) {
                if (err) *err = {attrs[i].location, it->second, attrs[i].format};
                return fail(ZR_ERROR_DUPLICATE_VERTEX_ATTRIBUTE_LOCATION,
                            "duplicate vertex attribute location: " + std::to_string(attrs[i].location));
            }
        } else {
            provided[attrs[i].location] = attrs[i].format;
        }
    }
    for (const auto& kv : expected) {
        auto it = provided.find(kv.first);
        if (it == provided.end()) {
            if (err) *err = {kv.first, kv.second, 0};
            return fail(ZR_ERROR_MISSING_VERTEX_ATTRIBUTE,
                        "missing vertex attribute for location " + std::to_string(kv.first));
        }
        if (it->second != kv.second) {
            if (err) *err = {kv.first, kv.second, it->second};
            return fail(ZR_ERROR_VERTEX_ATTRIBUTE_FORMAT_MISMATCH,
                        "vertex attribute format mismatch at location " + std::to_string(kv.first));
        }
    }
    for (const auto& kv : provided) {
        if (!expected.count(kv.first)) {
            if (err) *err = {kv.first, 0, kv.second};
            return fail(ZR_ERROR_UNEXPECTED_VERTEX_ATTRIBUTE,
                        "unexpected vertex attribute at location " + std::to_string(kv.first));
        }
    }
    return ZR_SUCCESS;
}

// The pipeline layout's push-constant ranges.  None given: one {ALL_GRAPHICS, 0,
// merged size} range when the size is > 0 (GraphicShaderInput::create_pipeline_layout,
// pipeline.rs:112-128).  Given: the VkPushConstantRange / VkPipelineLayoutCreateInfo
// valid usage (offset and size multiples of 4, size > 0, within
// maxPushConstantsSize, no stage in two ranges), and each stage's push-constant
// block [0, size) covered by ranges holding that stage (the pipeline's layout
// must match its shaders).
static zr_result push_constant_layout(const zr_graphic_pipeline_desc* desc, const zr_shader* vs, const zr_shader* fs,
                                      uint32_t merged, std::vector<zr_push_constant_range>& out) {
    out.clear();
    if (desc->push_constant_range_count == 0) {
        if (merged > kMaxPushBytes) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "push-constant block larger than 128 bytes");
        if (merged) out.push_back(zr_push_constant_range{ZR_SHADER_STAGE_ALL_GRAPHICS, 0u, merged});
        return ZR_SUCCESS;
    }
    if (!desc->push_constant_ranges) return fail(ZR_ERROR_VALIDATION_FAILED, "push_constant_ranges is NULL");
    uint32_t stages_seen = 0;
    for (uint32_t i = 0; i < desc->push_constant_range_count; ++i) {
        const zr_push_constant_range& r = desc->push_constant_ranges[i];
        if ((r.offset & 3u) || (r.size & 3u) || r.size == 0 || r.offset >= kMaxPushBytes || r.size > kMaxPushBytes - r.offset)
            return fail(ZR_ERROR_VALIDATION_FAILED, "push-constant range " + std::to_string(i) +
                                                        ": offset/size not multiples of 4, empty, or past 128 bytes");
        if (r.stage_flags == 0 || (r.stage_flags & ~(uint32_t)ZR_SHADER_STAGE_ALL_GRAPHICS))
            return fail(ZR_ERROR_VALIDATION_FAILED, "push-constant range " + std::to_string(i) + ": bad stage flags");
        if (stages_seen & r.stage_flags)
            return fail(ZR_ERROR_VALIDATION_FAILED, "a shader stage is in more than one push-constant range");
        stages_seen |= r.stage_flags;
        out.push_back(r);
    }
    for (const zr_shader* sh : {vs, fs}) {
        if (!sh || sh->push_constant_size == 0) continue;
        for (uint32_t w = 0; w < sh->push_constant_size / 4u; ++w) {
            bool covered = false;
            for (const auto& r : out)
                covered = covered || ((r.stage_flags & sh->stage) && w * 4u >= r.offset && w * 4u < r.offset + r.size);
            if (!covered)
                return fail(ZR_ERROR_VALIDATION_FAILED, "the layout's push-constant ranges do not cover the " +
                                                            std::string(sh->stage == ZR_SHADER_STAGE_VERTEX ? "vertex" : "fragment") +
                                                            " stage's push-constant block");
        }
    }
    return ZR_SUCCESS;
}

ZR_API zr_result zr_pipeline_create(zr_device* d, const zr_graphic_pipeline_desc* desc, zr_pipeline** out,
                                    zr_pipeline_error* err) {
    (void)d;
    if (!desc || !out) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    *out = nullptr;
    if (err) *err = {0, 0, 0};
    const zr_shader* vs = desc->vertex_shader;
    const zr_shader* fs = desc->fragment_shader;
    if (!vs) return fail(ZR_ERROR_MISSING_VERTEX_SHADER, "missing vertex shader");
    if (vs->stage != ZR_SHADER_STAGE_VERTEX || (fs && fs->stage != ZR_SHADER_STAGE_FRAGMENT))
        return fail(ZR_ERROR_VALIDATION_FAILED, "shader stage mismatch");
    zr_result rc = validate_vertex_inputs(vs, desc->vertex_attributes, desc->vertex_attribute_count, err);
    if (rc) return rc;
    if (fs && fs->program != vs->program)
        return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "vertex and fragment stages come from different programs");
    if (desc->topology != 3) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "only TRIANGLE_LIST is supported");
    if (desc->rasterization.polygon_mode != 0) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "only FILL polygon mode");
    if (desc->rasterization.depth_clamp || desc->rasterization.depth_bias_enable)
        return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "depth clamp / depth bias not supported");
    if (desc->samples > 1) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "only 1x multisampling");
    if (desc->color_attachment_count > 1) return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "at most one colour attachment");
    zr_pipeline* p = new (std::nothrow) zr_pipeline_t();
    if (!p) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "pipeline alloc");
    p->program = vs->program;
    p->has_fs = fs != nullptr;
    p->color_count = desc->color_attachment_count;
    p->color = zr_color_attachment_desc{};
    p->color.write_mask = 0xF;
    p->color_format = 0;
    if (p->color_count) {
        p->color = desc->color_attachments[0];
        p->color_format = desc->color_formats ? desc->color_formats[0] : 0;
        if (p->color.blend_enable) {
            delete p;
            return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "colour blending is not supported on this path");
        }
        if (p->color_format && format_bpp(p->color_format) == 0) {
            delete p;
            return fail(ZR_ERROR_FORMAT_NOT_SUPPORTED, "colour attachment format");
        }
    }
    p->depth_format = desc->depth_format;
    p->has_depth_state = desc->depth_stencil != nullptr;
    if (p->has_depth_state) {
        p->ds = *desc->depth_stencil;
        if (p->ds.stencil_test_enable || p->ds.depth_bounds_test_enable) {
            delete p;
            return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "stencil / depth-bounds tests are not supported");
        }
        if (p->ds.depth_write_enable && p->ds.depth_test_enable && p->ds.depth_compare_op == 5) {
            delete p;
            return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "NOT_EQUAL with depth writes is order dependent");
        }
    }
    p->cull_mode = desc->rasterization.cull_mode;
    p->front_face = desc->rasterization.front_face;
    // vertex layout: binding 0, per-vertex rate (VertexLayout derive, rhi-derive/src/lib.rs:126-131)
    p->stride = 0;
    for (uint32_t i = 0; i < desc->vertex_binding_count; ++i) {
        if (desc->vertex_bindings[i].binding == 0) {
            p->stride = desc->vertex_bindings[i].stride;
            if (desc->vertex_bindings[i].input_rate != 0) {
                delete p;
                return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "per-instance vertex input rate");
            }
        }
    }
    p->nattr = (uint32_t)vs->inputs.size();
    memset(p->attr_offset, 0, sizeof p->attr_offset);
    memset(p->attr_size, 0, sizeof p->attr_size);
    for (uint32_t i = 0; i < desc->vertex_attribute_count; ++i) {
        const auto& a = desc->vertex_attributes[i];
        if (a.binding != 0 || a.location >= 4 || (a.offset & 3u)) {
            delete p;
            return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "vertex attributes must live in binding 0, 4-byte aligned");
        }
        p->attr_offset[a.location] = a.offset;
        p->attr_size[a.location] = a.format == ZR_FORMAT_R32G32_SFLOAT ? 8u : a.format == ZR_FORMAT_R32_SFLOAT ? 4u
                                   : a.format == ZR_FORMAT_R32G32B32A32_SFLOAT ? 16u : 12u;
    }
    if (p->nattr && (p->stride == 0 || (p->stride & 3u))) {
        delete p;
        return fail(ZR_ERROR_FEATURE_NOT_PRESENT, "vertex binding 0 missing or stride not 4-byte aligned");
    }
    // ShaderReflection::merge (shader.rs:222-259): union by (set, binding), stage flags OR-ed
    std::map<std::pair<uint32_t, uint32_t>, zr_shader_binding> merged;
    for (const zr_shader* sh : {vs, fs}) {
        if (!sh) continue;
        for (const auto& b : sh->bindings) {
            auto key = std::make_pair(b.set, b.binding);
            auto it = merged.find(key);
            if (it == merged.end()) merged[key] = b;
            else it->second.stage_flags |= b.stage_flags;
        }
    }
    for (const auto& kv : merged) p->bindings.push_back(kv.second);
    // push constants: the merged size (the max over the stages, shader.rs:224-228)
    // and the layout's ranges -- derived as create_pipeline_layout does
    // (pipeline.rs:112-128), or the caller's, validated
    p->push_size = std::max(vs->push_constant_size, fs ? fs->push_constant_size : 0u);
    if ((rc = push_constant_layout(desc, vs, fs, p->push_size, p->push_ranges))) {
        delete p;
        return rc;
    }
    p->view_push = p->program == kProgMesh && vs->push_constant_size >= 64u;
    *out = p;
    return ZR_SUCCESS;
}

ZR_API void zr_pipeline_destroy(zr_pipeline* p) { delete p; }

ZR_API int32_t zr_pipeline_push_constant_ranges(const zr_pipeline* p, zr_push_constant_range* out, int32_t capacity) {
    if (!p) return 0;
    const int32_t n = (int32_t)p->push_ranges.size();
    for (int32_t i = 0; out && i < std::min(n, capacity); ++i) out[i] = p->push_ranges[i];
    return n;
}

// ----------------------------------------------------------------- commands

ZR_API zr_result zr_cmd_create(zr_device* d, zr_cmd** out) {
    // d may be NULL: a list recorded without a device (host-side validation of the
    // recording calls, e.g. on a machine without a GPU); zr_submit rejects it
    if (!out) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    zr_cmd* c = new (std::nothrow) zr_cmd_t();
    if (!c) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "cmd alloc");
    c->dev = d;
    *out = c;
    return ZR_SUCCESS;
}

ZR_API void zr_cmd_destroy(zr_cmd* c) {
    if (!c) return;
    if (c->dev) {
        auto& pend = c->dev->pending;
        if (std::find(pend.begin(), pend.end(), c) != pend.end()) device_sync(c->dev);
    }
    c->drop_graph();
    delete c;
}

ZR_API zr_result zr_cmd_begin(zr_cmd* c) {
    if (!c) return fail(ZR_ERROR_VALIDATION_FAILED, "cmd is NULL");
    if (c->dev) {
        auto& pend = c->dev->pending;
        if (std::find(pend.begin(), pend.end(), c) != pend.end()) {
            zr_result rc = device_sync(c->dev);
            if (rc) return rc;
        }
    }
    c->cmds.clear();
    c->push_data.clear();
    c->err = ZR_SUCCESS;
    c->err_msg.clear();
    c->in_rendering = false;
    c->drop_graph();
    c->eager_runs = 0;
    c->has_exchange = false;
    return ZR_SUCCESS;
}

ZR_API zr_result zr_cmd_end(zr_cmd* c) {
    if (!c) return fail(ZR_ERROR_VALIDATION_FAILED, "cmd is NULL");
    if (c->in_rendering) latch(c, ZR_ERROR_VALIDATION_FAILED, "command buffer ended inside a render pass");
    if (c->err) return fail(c->err, c->err_msg);
    return ZR_SUCCESS;
}

ZR_API void zr_cmd_begin_rendering(zr_cmd* c, const zr_rendering_info* info) {
    if (!c) return;
    if (!info) return latch(c, ZR_ERROR_VALIDATION_FAILED, "rendering info is NULL");
    if (c->in_rendering) return latch(c, ZR_ERROR_VALIDATION_FAILED, "nested begin_rendering");
    if (info->color_attachment_count > 1)
        return latch(c, ZR_ERROR_FEATURE_NOT_PRESENT, "at most one colour attachment");
    Cmd k;
    k.type = C_BEGIN_RENDERING;
    k.rendering.area = info->render_area;
    if (info->color_attachment_count == 1) {
        k.rendering.has_color = info->color_attachments[0].texture != nullptr;
        k.rendering.color = info->color_attachments[0];
    }
    if (info->depth_attachment && info->depth_attachment->texture) {
        k.rendering.has_depth = true;
        k.rendering.depth = *info->depth_attachment;
    }
    c->cmds.push_back(k);
    c->in_rendering = true;
}

ZR_API void zr_cmd_end_rendering(zr_cmd* c) {
    if (!c) return;
    if (!c->in_rendering) return latch(c, ZR_ERROR_VALIDATION_FAILED, "end_rendering without begin_rendering");
    Cmd k;
    k.type = C_END_RENDERING;
    c->cmds.push_back(k);
    c->in_rendering = false;
}

ZR_API void zr_cmd_clear_color_image(zr_cmd* c, zr_texture* t, const float clear_value[4]) {
    if (!c) return;
    if (c->in_rendering) return latch(c, ZR_ERROR_VALIDATION_FAILED, "clear_color_image inside a render pass");
    if (!t || !clear_value) return latch(c, ZR_ERROR_VALIDATION_FAILED, "clear_color_image: NULL argument");
    if (t->format == ZR_FORMAT_D32_SFLOAT) return latch(c, ZR_ERROR_VALIDATION_FAILED, "clear_color_image on a depth texture");
    Cmd k;
    k.type = C_CLEAR_IMAGE;
    k.rendering.area = zr_rect2d{0, 0, t->width, t->height};
    k.rendering.has_color = true;
    k.rendering.color.texture = t;
    k.rendering.color.load_op = ZR_ATTACHMENT_LOAD_OP_CLEAR;
    for (int i = 0; i < 4; ++i) k.rendering.color.clear_value[i] = clear_value[i];
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_bind_pipeline(zr_cmd* c, const zr_pipeline* p) {
    if (!c) return;
    if (!p) return latch(c, ZR_ERROR_VALIDATION_FAILED, "pipeline is NULL");
    Cmd k;
    k.type = C_BIND_PIPELINE;
    k.pipeline = p;
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_bind_uniform_buffer(zr_cmd* c, uint32_t set, uint32_t binding, const zr_buffer* buf,
                                       uint64_t offset, uint64_t range) {
    if (!c) return;
    if (!buf) return latch(c, ZR_ERROR_VALIDATION_FAILED, "uniform buffer is NULL");
    Cmd k;
    k.type = C_BIND_UNIFORM;
    k.a = set;
    k.b = binding;
    k.buffer = buf;
    k.offset = offset;
    k.range = range;
    c->cmds.push_back(k);
}

ZR_API zr_result zr_cmd_bind_uniform_by_name(zr_cmd* c, const zr_pipeline* p, const char* name, const zr_buffer* buf,
                                             uint64_t offset, uint64_t range) {
    if (!c || !p || !name || !buf) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    for (const auto& b : p->bindings) {
        if (!strcmp(b.name, name)) {
            if (b.descriptor_type != ZR_DESCRIPTOR_TYPE_UNIFORM_BUFFER && b.descriptor_type != ZR_DESCRIPTOR_TYPE_STORAGE_BUFFER)
                return fail(ZR_ERROR_BINDING_TYPE_MISMATCH, std::string("binding '") + name + "' is not a buffer");
            zr_cmd_bind_uniform_buffer(c, b.set, b.binding, buf, offset, range);
            return ZR_SUCCESS;
        }
    }
    return fail(ZR_ERROR_BINDING_NOT_FOUND, std::string("binding '") + name + "' not found");
}

ZR_API void zr_cmd_push_constants(zr_cmd* c, const zr_pipeline* layout, uint32_t stage_flags, uint32_t offset,
                                  uint32_t size, const void* data) {
    if (!c) return;
    if (!layout || !data) return latch(c, ZR_ERROR_VALIDATION_FAILED, "push_constants: NULL layout or data");
    if ((offset & 3u) || (size & 3u) || size == 0 || offset >= kMaxPushBytes || size > kMaxPushBytes - offset)
        return latch(c, ZR_ERROR_VALIDATION_FAILED,
                     "push_constants: offset/size not multiples of 4, empty, or past maxPushConstantsSize (128)");
    if (stage_flags == 0) return latch(c, ZR_ERROR_VALIDATION_FAILED, "push_constants: no stage flags");
    // VUID-vkCmdPushConstants-offset-01795 / -01796: every byte of the update lies in
    // a range holding every stage of stage_flags, and stage_flags holds every stage
    // of each range the update overlaps
    for (uint32_t b = offset; b < offset + size; b += 4u) {
        uint32_t stages = 0;
        for (const auto& r : layout->push_ranges) {
            if (b < r.offset || b >= r.offset + r.size) continue;
            stages |= r.stage_flags;
            if ((r.stage_flags & stage_flags) != r.stage_flags)
                return latch(c, ZR_ERROR_VALIDATION_FAILED,
                             "push_constants: stage_flags miss a stage of a push-constant range the update overlaps");
        }
        if ((stages & stage_flags) != stage_flags)
            return latch(c, ZR_ERROR_VALIDATION_FAILED,
                         "push_constants: bytes outside the layout's push-constant ranges for these stages");
    }
    Cmd k;
    k.type = C_PUSH_CONSTANTS;
    k.pipeline = layout;
    k.a = offset;
    k.b = size;
    k.offset = c->push_data.size();
    c->push_data.insert(c->push_data.end(), (const uint8_t*)data, (const uint8_t*)data + size);
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_set_viewport(zr_cmd* c, uint32_t first, uint32_t count, const zr_viewport* vps) {
    if (!c) return;
    if (!vps || count == 0) return;
    if (first != 0 || count != 1) return latch(c, ZR_ERROR_FEATURE_NOT_PRESENT, "only viewport 0");
    Cmd k;
    k.type = C_SET_VIEWPORT;
    k.vp = vps[0];
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_set_scissor(zr_cmd* c, uint32_t first, uint32_t count, const zr_rect2d* rects) {
    if (!c) return;
    if (!rects || count == 0) return;
    if (first != 0 || count != 1) return latch(c, ZR_ERROR_FEATURE_NOT_PRESENT, "only scissor 0");
    Cmd k;
    k.type = C_SET_SCISSOR;
    k.rect = rects[0];
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_bind_vertex_buffers(zr_cmd* c, uint32_t first_binding, uint32_t count, const zr_buffer* const* bufs,
                                       const uint64_t* offsets) {
    if (!c) return;
    for (uint32_t i = 0; i < count; ++i) {
        if (!bufs || !bufs[i]) return latch(c, ZR_ERROR_VALIDATION_FAILED, "vertex buffer is NULL");
        Cmd k;
        k.type = C_BIND_VB;
        k.a = first_binding + i;
        k.buffer = bufs[i];
        k.offset = offsets ? offsets[i] : 0;
        c->cmds.push_back(k);
    }
}

ZR_API void zr_cmd_bind_index_buffer(zr_cmd* c, const zr_buffer* buf, uint64_t offset, int32_t index_type) {
    if (!c) return;
    if (!buf) return latch(c, ZR_ERROR_VALIDATION_FAILED, "index buffer is NULL");
    if (index_type != ZR_INDEX_TYPE_UINT16 && index_type != ZR_INDEX_TYPE_UINT32)
        return latch(c, ZR_ERROR_FEATURE_NOT_PRESENT, "index type");
    Cmd k;
    k.type = C_BIND_IB;
    k.buffer = buf;
    k.offset = offset;
    k.e = index_type;
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_draw(zr_cmd* c, uint32_t vertex_count, uint32_t instance_count, uint32_t first_vertex,
                        uint32_t first_instance) {
    if (!c) return;
    Cmd k;
    k.type = C_DRAW;
    k.a = vertex_count;
    k.b = instance_count;
    k.c = first_vertex;
    k.d = 0;
    k.e = 0;
    (void)first_instance;
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_draw_indexed(zr_cmd* c, uint32_t index_count, uint32_t instance_count, uint32_t first_index,
                                int32_t vertex_offset, uint32_t first_instance) {
    if (!c) return;
    Cmd k;
    k.type = C_DRAW;
    k.a = index_count;
    k.b = instance_count;
    k.c = first_index;
    k.d = 1;
    k.e = vertex_offset;
    (void)first_instance;
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_set_tile_shard(zr_cmd* c, uint32_t rank, uint32_t count) {
    if (!c) return;
    if (count == 0 || rank >= count) return latch(c, ZR_ERROR_VALIDATION_FAILED, "bad tile shard");
    Cmd k;
    k.type = C_SET_SHARD;
    k.a = rank;
    k.b = count;
    c->cmds.push_back(k);
}

ZR_API void zr_cmd_set_tile_shard_exchange(zr_cmd* c, uint32_t rank, uint32_t count, zr_exchange_fn exchange,
                                           void* user) {
    if (!c) return;
    if (count == 0 || rank >= count || count > kMaxShards) return latch(c, ZR_ERROR_VALIDATION_FAILED, "bad tile shard");
    if (!exchange) return latch(c, ZR_ERROR_VALIDATION_FAILED, "tile shard exchange is NULL");
    Cmd k;
    k.type = C_SET_SHARD;
    k.a = rank;
    k.b = count;
    k.exchange = exchange;
    k.exchange_user = user;
    c->cmds.push_back(k);
    c->has_exchange = true;
}

ZR_API void zr_cmd_set_route_capacity(zr_cmd* c, uint32_t entries) {
    if (!c) return;
    Cmd k;
    k.type = C_SET_ROUTE_CAP;
    k.a = entries;
    c->cmds.push_back(k);
}

// ------------------------------------------------------------ multi-GPU (RCCL)

namespace {

// The built-in zr_exchange_fn: one grouped send + receive per rank over the
// device's exchange communicator, enqueued on the stream the runtime passes.
zr_result rccl_exchange(void* user, void* stream, const void* send, void* recv, uint64_t bytes_per_rank) {
    zr_device* d = (zr_device*)user;
    if (!d || !d->comm_x) return fail(ZR_ERROR_INITIALIZATION_FAILED, "zr_rccl_exchange_fn: device has no RCCL communicator");
    std::string err;
    const hipStream_t s = (hipStream_t)stream;
    if (rccl_has_all_to_all()) {
        if (!rccl_all_to_all(send, recv, bytes_per_rank, d->comm_x, s, err)) return fail(ZR_ERROR_DEVICE_LOST, err);
        return ZR_SUCCESS;
    }
    zr_transfer_op plan[2 * kMaxShards];
    const int32_t n = zr_exchange_plan(d->comm_size, d->comm_rank, bytes_per_rank, plan, 2 * (int32_t)kMaxShards);
    if (n < 0) return fail(ZR_ERROR_VALIDATION_FAILED, "bad exchange plan (rank / rank count)");
    P2POp ops[2 * kMaxShards];
    for (int32_t i = 0; i < n; ++i)
        ops[i] = P2POp{plan[i].send ? (void*)((const uint8_t*)send + plan[i].offset) : (void*)((uint8_t*)recv + plan[i].offset),
                       (size_t)plan[i].bytes, plan[i].peer, plan[i].send != 0};
    if (!rccl_grouped(ops, (size_t)n, d->comm_x, s, err)) return fail(ZR_ERROR_DEVICE_LOST, err);
    return ZR_SUCCESS;
}

}  // namespace

// Host-side plans of the two collectives (no device needed; tests/test_abi.py).
// Gather (ShardGeom ownership): a round-robin tile row is a contiguous span of the
// linear image, sent from its owner straight into place on the root; a leftover
// row holds one run of tiles per owner, a rectangle (rows spans `pitch` apart)
// unless it is the whole row -- the runtime packs it into a staging buffer to send
// and unpacks it on the root.  One op per (tile row, owner), none for the root's
// own tiles.  `offset` is the byte offset in the image (the same on both sides);
// the last tile row may be partial.
ZR_API uint32_t zr_tile_size(void) { return (uint32_t)kTile; }

ZR_API int32_t zr_gather_plan(uint32_t width, uint32_t height, uint32_t bytes_per_pixel, int32_t nranks, int32_t rank,
                              int32_t root, zr_transfer_op* out, int32_t capacity) {
    if (nranks < 1 || nranks > (int32_t)kMaxShards || rank < 0 || rank >= nranks || root < 0 || root >= nranks ||
        width == 0 || height == 0 || bytes_per_pixel == 0)
        return -1;
    const uint32_t tiles_x = (width + kTile - 1) / kTile, tiles_y = (height + kTile - 1) / kTile;
    const uint64_t row_bytes = (uint64_t)width * bytes_per_pixel;
    int32_t n = 0;
    auto emit = [&](int32_t owner, uint32_t ty, uint32_t c0, uint32_t c1) {  // tiles [c0, c1] of row ty
        if (owner == root || (rank != root && rank != owner)) return;
        const uint32_t rows = std::min<uint32_t>(kTile, height - ty * kTile);
        const uint32_t x0 = c0 * kTile, x1 = std::min<uint32_t>(width, (c1 + 1) * kTile);
        if (out && n < capacity) {
            zr_transfer_op& op = out[n];
            memset(&op, 0, sizeof op);
            op.peer = rank == root ? owner : root;
            op.send = rank == root ? 0 : 1;
            op.offset = (uint64_t)ty * kTile * row_bytes + (uint64_t)x0 * bytes_per_pixel;
            if (x0 == 0 && x1 == width) {  // whole rows: one contiguous span
                op.bytes = (uint64_t)rows * row_bytes;
                op.rows = 1;
            } else {
                op.bytes = (uint64_t)(x1 - x0) * bytes_per_pixel;
                op.rows = rows;
                op.pitch = row_bytes;
            }
        }
        ++n;
    };
    for (int32_t r = 0; r < nranks; ++r) {
        const ShardGeom sg = shard_geom(tiles_x, tiles_y, (uint32_t)nranks, (uint32_t)r);
        for (uint32_t ty = (uint32_t)r; ty < sg.full_rows; ty += (uint32_t)nranks) emit(r, ty, 0, tiles_x - 1);
        for (uint32_t i = sg.left_lo; i < sg.left_hi;) {  // its leftover run, cut at row ends
            const uint32_t ty = sg.full_rows + i / tiles_x, c0 = i % tiles_x;
            const uint32_t c1 = std::min(tiles_x - 1, c0 + (sg.left_hi - i) - 1);
            emit(r, ty, c0, c1);
            i += c1 - c0 + 1;
        }
    }
    return n;
}

// Exchange (all-to-all without ncclAllToAll): to every rank p (itself included)
// send block p of the send buffer, and receive p's block for this rank at p *
// bytes_per_rank of the receive buffer, paired per peer in one group.
ZR_API int32_t zr_exchange_plan(int32_t nranks, int32_t rank, uint64_t bytes_per_rank, zr_transfer_op* out,
                                int32_t capacity) {
    if (nranks < 1 || nranks > (int32_t)kMaxShards || rank < 0 || rank >= nranks) return -1;
    int32_t n = 0;
    for (int32_t p = 0; p < nranks; ++p)
        for (int32_t send = 1; send >= 0; --send) {
            if (out && n < capacity) {
                memset(&out[n], 0, sizeof out[n]);
                out[n].peer = p;
                out[n].send = send;
                out[n].offset = (uint64_t)p * bytes_per_rank;
                out[n].bytes = bytes_per_rank;
                out[n].rows = 1;
            }
            ++n;
        }
    return n;
}

ZR_API int32_t zr_rccl_available(void) {
    std::string err;
    return rccl_load(err) ? 1 : 0;
}

ZR_API zr_result zr_rccl_get_unique_id(void* out) {
    if (!out) return fail(ZR_ERROR_VALIDATION_FAILED, "out is NULL");
    std::string err;
    if (!rccl_unique_id(out, err)) return fail(ZR_ERROR_INITIALIZATION_FAILED, err);
    return ZR_SUCCESS;
}

ZR_API zr_result zr_device_init_rccl(zr_device* d, const void* exchange_id, const void* gather_id, int32_t nranks,
                                     int32_t rank) {
    if (!d || !exchange_id || !gather_id) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    if (nranks < 1 || nranks > (int32_t)kMaxShards || rank < 0 || rank >= nranks)
        return fail(ZR_ERROR_VALIDATION_FAILED, "bad rank / rank count");
    if (d->comm_x) return fail(ZR_ERROR_VALIDATION_FAILED, "device already has RCCL communicators");
    zr_result rc = set_device(d);
    if (rc) return rc;
    std::string err;
    if (!rccl_comm_init(&d->comm_x, exchange_id, nranks, rank, err) ||
        !rccl_comm_init(&d->comm_g, gather_id, nranks, rank, err)) {
        rccl_comm_destroy(d->comm_x);
        d->comm_x = nullptr;
        return fail(ZR_ERROR_INITIALIZATION_FAILED, err);
    }
    d->comm_rank = rank;
    d->comm_size = nranks;
    ZR_HIP(hipStreamCreateWithFlags(&d->gather_stream, hipStreamNonBlocking));
    ZR_HIP(hipEventCreateWithFlags(&d->frame_done, hipEventDisableTiming));
    return ZR_SUCCESS;
}

ZR_API zr_exchange_fn zr_rccl_exchange_fn(void) { return &rccl_exchange; }

namespace {

// The recorded receive blocks must be whole blocks of this draw's layout: the
// receive buffer holds shard_count x bytes_per_rank bytes (exec_draw checks the
// count against the draw before the route runs; here, without the count, a size
// that is no whole number of blocks or more than kMaxShards of them is refused --
// a buffer recorded at another route capacity or shard count would otherwise be
// copied past the end of the receive buffer).
zr_result replay_exchange(void* user, void* stream, const void* send, void* recv, uint64_t bytes_per_rank) {
    (void)send;
    const zr_replay_exchange* r = (const zr_replay_exchange*)user;
    if (!r || !r->src) return fail(ZR_ERROR_VALIDATION_FAILED, "zr_replay_exchange_fn: no recorded buffer");
    if (bytes_per_rank == 0 || r->bytes == 0 || r->bytes % bytes_per_rank != 0 || r->bytes / bytes_per_rank > kMaxShards)
        return fail(ZR_ERROR_VALIDATION_FAILED,
                    "zr_replay_exchange_fn: recorded bytes are not whole exchange blocks of this draw's layout");
    ZR_HIP(hipMemcpyAsync(recv, r->src, r->bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return ZR_SUCCESS;
}

}  // namespace

ZR_API zr_exchange_fn zr_replay_exchange_fn(void) { return &replay_exchange; }

ZR_API zr_result zr_device_gather_tile_rows(zr_device* d, zr_texture* t, int32_t root) {
    if (!d || !t) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    if (!d->comm_g) return fail(ZR_ERROR_INITIALIZATION_FAILED, "device has no RCCL communicator (zr_device_init_rccl)");
    if (root < 0 || root >= d->comm_size) return fail(ZR_ERROR_VALIDATION_FAILED, "bad root rank");
    zr_result rc = set_device(d);
    if (rc) return rc;
    if (!t->gather_done) ZR_HIP(hipEventCreateWithFlags(&t->gather_done, hipEventDisableTiming));
    // after everything enqueued so far on the device stream (the frame)
    ZR_HIP(hipEventRecord(d->frame_done, d->stream));
    ZR_HIP(hipStreamWaitEvent(d->gather_stream, d->frame_done, 0));
    const int32_t n = zr_gather_plan(t->width, t->height, t->bpp, d->comm_size, d->comm_rank, root, nullptr, 0);
    std::vector<zr_transfer_op> plan((size_t)std::max(n, 0));
    zr_gather_plan(t->width, t->height, t->bpp, d->comm_size, d->comm_rank, root, plan.data(), n);
    // rectangles (leftover rows' tile runs) travel packed through a staging buffer
    uint64_t stage_bytes = 0;
    for (const zr_transfer_op& op : plan)
        if (op.rows > 1) stage_bytes += op.bytes * op.rows;
    if (stage_bytes > d->gather_stage_cap) {
        ZR_HIP(hipStreamSynchronize(d->gather_stream));
        if (d->gather_stage) ZR_HIP(hipFree(d->gather_stage));
        d->gather_stage = nullptr;
        ZR_HIP(hipMalloc((void**)&d->gather_stage, stage_bytes));
        d->gather_stage_cap = stage_bytes;
    }
    const hipStream_t gs = d->gather_stream;
    uint64_t so = 0;
    for (const zr_transfer_op& op : plan) {  // senders pack first
        if (op.rows <= 1) continue;
        if (op.send)
            ZR_HIP(hipMemcpy2DAsync(d->gather_stage + so, op.bytes, (const uint8_t*)t->ptr + op.offset, op.pitch, op.bytes,
                                    op.rows, hipMemcpyDeviceToDevice, gs));
        so += op.bytes * op.rows;
    }
    std::string err;
    std::vector<P2POp> ops;
    ops.reserve(plan.size());
    so = 0;
    for (const zr_transfer_op& op : plan) {
        uint8_t* p = (uint8_t*)t->ptr + op.offset;
        uint64_t bytes = op.bytes;
        if (op.rows > 1) {
            p = d->gather_stage + so;
            bytes = op.bytes * op.rows;
            so += bytes;
        }
        ops.push_back(P2POp{p, (size_t)bytes, op.peer, op.send != 0});
    }
    // one balanced group (rccl_grouped: no ncclGroupEnd after a failed start)
    if (!rccl_grouped(ops.data(), ops.size(), d->comm_g, gs, err)) return fail(ZR_ERROR_DEVICE_LOST, err);
    so = 0;
    for (const zr_transfer_op& op : plan) {  // the root unpacks after the group
        if (op.rows <= 1) continue;
        if (!op.send)
            ZR_HIP(hipMemcpy2DAsync((uint8_t*)t->ptr + op.offset, op.pitch, d->gather_stage + so, op.bytes, op.bytes,
                                    op.rows, hipMemcpyDeviceToDevice, gs));
        so += op.bytes * op.rows;
    }
    ZR_HIP(hipEventRecord(t->gather_done, d->gather_stream));
    t->gather_pending = true;
    return ZR_SUCCESS;
}

// --------------------------------------------------------------- submission

ZR_API zr_result zr_fence_create(zr_device* d, zr_fence** out) {
    if (!d || !out) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    zr_result rc = set_device(d);
    if (rc) return rc;
    zr_fence* f = new (std::nothrow) zr_fence_t();
    if (!f) return fail(ZR_ERROR_OUT_OF_HOST_MEMORY, "fence alloc");
    f->dev = d;
    if (hipEventCreateWithFlags(&f->ev, hipEventDisableTiming) != hipSuccess) {
        delete f;
        return fail(ZR_ERROR_DEVICE_LOST, "hipEventCreate failed");
    }
    *out = f;
    return ZR_SUCCESS;
}

ZR_API void zr_fence_destroy(zr_fence* f) {
    if (!f) return;
    (void)hipEventSynchronize(f->ev);
    (void)hipEventDestroy(f->ev);
    delete f;
}

// Executes a command list on the device stream.  The first submission runs eagerly
// (sizing scratch); the second captures the same launches into a HIP graph, later
// ones replay it (one launch per frame instead of one per kernel).
static zr_result submit_graph_or_eager(zr_device* d, zr_cmd* c) {
    const bool graphs = d->use_graphs && !d->profiling && !d->debug && !c->has_exchange;
    if (!graphs || c->eager_runs == 0) {
        c->eager_runs++;
        return execute(d, c);
    }
    // a replayed graph's draws read and write scratch set 0 on the main stream
    auto mark_set0 = [d]() -> zr_result {
        d->sets[0].main_reader_pending = true;
        return ZR_SUCCESS;
    };
    if (c->graph && c->graph_gen == d->scratch_gen) {
        ZR_HIP(hipGraphLaunch(c->graph, d->stream));
        return mark_set0();
    }
    c->drop_graph();
    const uint64_t gen = d->scratch_gen;
    ZR_HIP(hipStreamBeginCapture(d->stream, hipStreamCaptureModeRelaxed));
    d->capturing = true;
    zr_result rc = execute(d, c);
    d->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(d->stream, &g);
    if (rc == ZR_SUCCESS && e == hipSuccess && g && d->scratch_gen == gen) {
        const hipError_t ie = hipGraphInstantiate(&c->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ie == hipSuccess) {
            c->graph_gen = gen;
            ZR_HIP(hipGraphLaunch(c->graph, d->stream));
            return mark_set0();
        }
        c->graph = nullptr;
    } else if (g) {
        (void)hipGraphDestroy(g);
    }
    if (rc != ZR_SUCCESS && rc != ZR_NOT_READY) return rc;
    c->eager_runs++;
    return execute(d, c);  // scratch had to grow (or capture failed): run eagerly
}

ZR_API zr_result zr_submit(zr_device* d, zr_cmd* c, zr_fence* f) {
    if (!d || !c) return fail(ZR_ERROR_VALIDATION_FAILED, "NULL argument");
    if (c->dev != d) return fail(ZR_ERROR_VALIDATION_FAILED, "command list was created for another device (or none)");
    if (c->err) return fail(c->err, c->err_msg);
    if (c->in_rendering) return fail(ZR_ERROR_VALIDATION_FAILED, "submitted inside a render pass");
    zr_result rc = set_device(d);
    if (rc) return rc;
    rc = submit_graph_or_eager(d, c);
    if (rc) return rc;
    if (std::find(d->pending.begin(), d->pending.end(), c) == d->pending.end()) d->pending.push_back(c);
    if (f) {
        ZR_HIP(hipEventRecord(f->ev, d->stream));
        f->submitted = true;
    }
    return ZR_SUCCESS;
}

ZR_API zr_result zr_fence_wait(zr_fence* f, uint64_t timeout_ns) {
    if (!f) return fail(ZR_ERROR_VALIDATION_FAILED, "fence is NULL");
    if (!f->submitted) return ZR_SUCCESS;
    if (timeout_ns == 0) {
        hipError_t e = hipEventQuery(f->ev);
        if (e == hipErrorNotReady) return ZR_TIMEOUT;
        if (e != hipSuccess) return fail(ZR_ERROR_DEVICE_LOST, hipGetErrorString(e));
    }
    return device_sync(f->dev);
}

ZR_API zr_result zr_submit_and_wait(zr_device* d, zr_cmd* c) {
    zr_result rc = zr_submit(d, c, nullptr);
    if (rc) return rc;
    return device_sync(d);
}

}  // extern "C"
