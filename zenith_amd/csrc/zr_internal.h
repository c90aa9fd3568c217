// zr_internal.h — data layout shared by the host runtime and the HIP kernels.
// DESIGN.md §4 describes each buffer's HBM layout and the per-unit byte counts.
#pragma once
#include <stdint.h>

#include <algorithm>

namespace zr {

// Screen tiles (one k_tile workgroup per tile) are 16, 32 or 64 pixels on a side,
// chosen per draw (DrawParams::tile_shift, tile_shift_for below).
// 32 is the default and the unit of tile-row shard ownership, of the row gather
// and of k_clear; zr_tile_size() reports it and zenith_amd/shard.py reads it there.
constexpr int kTile = 32;
constexpr int kTileShift = 5;
constexpr int kTilePixels = kTile * kTile;
constexpr uint32_t kTileShiftMin = 4, kTileShiftMax = 6;
constexpr int kTileThreads = 256;  // k_tile workgroup: 4 waves of 64 (512 for some passes: tile_threads_for)
constexpr uint32_t kSortCap = 1024;     // tile-list segment sorted by area in LDS
constexpr uint32_t kBigQueue = 512;     // k_tile: queued wave-path primitives per segment
constexpr uint32_t kSortBuckets = 64;   // cost classes: the lane walk's pair steps over bbox ∩ tile, min((steps - 1) >> 1, 63)
constexpr int kSetupThreads = 1024;  // setup / bin workgroups (one LDS histogram each)
constexpr uint32_t kSetupLdsBudget = 160u * 1024u;     // one k_setup_bin workgroup per CU owns the LDS
constexpr uint32_t kSetupBboxLdsBytes = 96u * 1024u;  // cap on the per-workgroup bbox array in LDS
#ifndef ZR_BIN_STAGE_DEFAULT
#define ZR_BIN_STAGE_DEFAULT 1
#endif
constexpr bool kBinStageDefault = ZR_BIN_STAGE_DEFAULT;  // k_setup_bin phase 4 staged in LDS (ZR_BIN_STAGE)

enum Program : int32_t { kProgTriangle = 0, kProgFlat = 1, kProgBlinn = 2, kProgMesh = 3, kProgCount = 4 };

// The mesh program (camera + clipping) cuts a primitive against
// the depth planes into a fan of up to 3 triangles.  Fan k > 0 of primitive p
// has setup record prims + 2p + k - 1 (records are sized 3 * prims); every fan
// triangle of p carries the visibility sequence 4p + k + 1 (API order; fans of
// one primitive never overlap).
constexpr uint32_t kMeshFans = 3;

// Visibility-key schemes: the per-pixel 64-bit atomicMin key
// reproduces in-order Vulkan depth-test semantics independent of fragment order.
enum DepthMode : int32_t {
    kDepthLastWins = 0,     // no depth write (or ALWAYS/EQUAL): pre-test vs initial depth, last primitive wins
    kDepthMinStrict = 1,    // LESS + write: min z, ties -> first
    kDepthMinNonStrict = 2, // LESS_OR_EQUAL + write: min z, ties -> last
    kDepthMaxStrict = 3,    // GREATER + write: max z, ties -> first
    kDepthMaxNonStrict = 4, // GREATER_OR_EQUAL + write: max z, ties -> last
    kDepthModeCount = 5,
};

// Per-primitive setup record, 64 B (4 x 16 B), written once by k_setup.
// Vertices are oriented so that A2 > 0 (v1/v2 swapped when needed; flag bit 0).
struct alignas(16) TriRecord {
    int32_t X0, Y0, X1, Y1;   // 24.8 fixed-point framebuffer coordinates
    int32_t X2, Y2;
    float z0, dz1;            // z0, z1 - z0
    float dz2, invA2;         // z2 - z0, 1 / (float)A2
    uint32_t v0, v1;          // vertex ids in record order (after the v1/v2 swap).  The built-in
    uint32_t v2;              // vertex stages emit w = 1 (triangle.slang:22), so 1/w = 1 and the
                              // perspective weights equal the barycentrics
    uint32_t bb0;             // px0 | py0 << 16  (inclusive pixel bbox, clipped)
    uint32_t bb1;             // px1 | py1 << 16
    uint32_t flags;           // bit0 swapped v1<->v2, bits1..3 edge bias (0 = top-left edge), bit4 small
};
static_assert(sizeof(TriRecord) == 64, "TriRecord must be 64 B");

// Compact per-primitive record, the one k_tile gathers for every (tile, primitive)
// pair: vertex 0 in 24.8 fixed point, vertices 1 and 2 as int16
// deltas from it (exact for kFlagSmall primitives: extents <= 64 px * 256), the
// depth terms, and 1/A2 with the orientation swap (kFlagSwapped) in its sign bit
// (A2 > 0 after orientation, so the bit is free).  Bias flags and the pixel bbox
// are recomputed from the vertices.  A primitive too large for int16 deltas has
// dx1 == kCompactLarge and its full TriRecord in records_big; its dy1 is 1 when it
// covers at most a quarter of its bbox (a sliver, which k_tile's lane walk takes
// in any cost bucket), else 0.
struct alignas(16) TriCompact {
    int32_t X0, Y0;
    int16_t dx1, dy1, dx2, dy2;
    float z0, dz1, dz2, invA2s;
};
static_assert(sizeof(TriCompact) == 32, "TriCompact must be 32 B");
constexpr int16_t kCompactLarge = -32768;

enum : uint32_t { kFlagSwapped = 1u, kFlagBias0 = 2u, kFlagBias1 = 4u, kFlagBias2 = 8u, kFlagSmall = 16u };
// A primitive is "small" when its fixed-point bbox spans <= 64 px in x and y: every
// edge function inside it then fits int32 (|w| <= 2^29), so the lane-parallel
// raster path steps edges incrementally in 32-bit integers.
constexpr int32_t kSmallExtent = 64 * 256;
constexpr uint32_t kEmptyBox = 0xFFFFFFFFu;
// Bin entry = setup record | cost class << kBinPrimBits, where the cost class is
// the lane walk's pair steps over bbox ∩ tile, ceil(w / 2) * h, as
// min((steps - 1) >> 1, kSortBuckets - 1) (k_setup_bin phase 4; k_tile sorts a
// tile's entries by it so that a 64-lane chunk holds walks of similar length).
constexpr uint32_t kBinPrimBits = 26;
constexpr uint32_t kBinPrimMask = (1u << kBinPrimBits) - 1u;
// k_setup_bin's cursor for a run the pool could not hold: its pairs are dropped
// (phase 4 stores only below 2^31; bin buffers stay under 2^30 entries) and the
// tile takes k_tile's record scan.
constexpr uint32_t kDropCursor = 0xC0000000u;
// run_counts[t] (DrawParams::runs): the slab fill in bits [9, 30) with kRunFill
// when a run straddled the slab end, kRunDropped when a run was dropped (bits
// [0, 9) unused).  Slabs are capped at kMaxSlab entries so the fill fits.
constexpr uint32_t kRunCountMask = 0x1FFu;
constexpr uint32_t kRunFillShift = 9;
constexpr uint32_t kMaxSlab = (1u << 21) - 1u;
constexpr uint32_t kRunFill = 1u << 30;
constexpr uint32_t kRunDropped = 1u << 31;
// tile_counts[t] bit 31: the tile has a pool run (set by k_setup_bin pool_run), so
// k_tile reads its run word -- a tile without one reads nothing more than its count
// (an extra load and reset store of the run word per tile: C3 tile pass +4 us)
constexpr uint32_t kCountRuns = 1u << 31;
constexpr uint32_t kMaxRunsPerTile = 256;  // k_tile keeps a tile's run table in its 512-word wave-path queue
struct alignas(8) BBox {
    uint32_t bb0, bb1;  // as TriRecord::bb0/bb1
};
constexpr uint32_t kMaxTilesPerPass = 16384;  // LDS histogram of the setup pass (64 KB)
constexpr uint32_t kJobTileBits = 14;          // tile_order item: tile | part << kJobTileBits (tiles < kMaxTilesPerPass)
constexpr uint32_t kJobTileMask = (1u << kJobTileBits) - 1u;
constexpr uint32_t kJobNone = 0xFFFFFFFFu;     // tile_order item of a spare block (job grids)
static_assert((1u << kJobTileBits) == kMaxTilesPerPass, "job items hold any tile index");
constexpr uint32_t kMaxPushBytes = 128;       // ZR_MAX_PUSH_CONSTANTS_SIZE (Vulkan's guaranteed minimum)
constexpr uint32_t kMaxPushWords = kMaxPushBytes / 4;

// Tile ownership of a G-way screen shard.  The first F =
// floor(tiles_y / G) * G tile rows go round robin, row ty to rank ty % G
// (interleaved for load balance); the tiles of the last tiles_y - F rows (n of
// them, row-major) are cut into G runs, rank r owning [ceil(r n / G), ceil((r + 1)
// n / G)) -- so every rank owns floor or ceil of all tiles / G (C2 at 1080p over 8
// ranks: 255 each instead of 5 or 4 rows of 60), and the tile of leftover index i
// belongs to rank floor(i G / n).  A rank's owned tiles are indexed round-robin
// rows first (own row o, column tx: o * tiles_x + tx), then its leftover run.
struct ShardGeom {
    uint32_t tiles_x, tiles_y, G, rank;
    uint32_t full_rows, own_rows, left_lo, left_hi;
};
__host__ __device__ inline ShardGeom shard_geom(uint32_t tiles_x, uint32_t tiles_y, uint32_t G, uint32_t rank) {
    ShardGeom s;
    s.tiles_x = tiles_x;
    s.tiles_y = tiles_y;
    s.G = G;
    s.rank = rank;
    s.own_rows = tiles_y / G;
    s.full_rows = s.own_rows * G;
    const uint64_t n = (uint64_t)(tiles_y - s.full_rows) * tiles_x;
    s.left_lo = (uint32_t)(((uint64_t)rank * n + G - 1) / G);
    s.left_hi = (uint32_t)(((uint64_t)(rank + 1) * n + G - 1) / G);
    return s;
}
__host__ __device__ inline uint32_t shard_tiles(const ShardGeom& s) {
    return s.own_rows * s.tiles_x + (s.left_hi - s.left_lo);
}
// Owner of tile (tx, ty).
__host__ __device__ inline uint32_t shard_owner(const ShardGeom& s, uint32_t tx, uint32_t ty) {
    if (ty < s.full_rows) return ty % s.G;
    const uint64_t n = (uint64_t)(s.tiles_y - s.full_rows) * s.tiles_x;
    return (uint32_t)(((uint64_t)(ty - s.full_rows) * s.tiles_x + tx) * s.G / n);
}
// Owned tile index t (< shard_tiles) -> tile coordinates.
__host__ __device__ inline void shard_tile_xy(const ShardGeom& s, uint32_t t, uint32_t& tx, uint32_t& ty) {
    const uint32_t fullc = s.own_rows * s.tiles_x;
    if (t < fullc) {
        const uint32_t o = t / s.tiles_x;
        tx = t - o * s.tiles_x;
        ty = o * s.G + s.rank;
    } else {
        const uint32_t i = s.left_lo + (t - fullc);
        ty = s.full_rows + i / s.tiles_x;
        tx = i % s.tiles_x;
    }
}

// Partitioned setup for tile-row shards.  Rank r sets up the
// primitives of its range [r * span, (r + 1) * span), kRouteChunk per workgroup
// of k_route, and ships each set-up primitive -- its compact record, pixel bbox
// and draw id -- to the ranks owning the tile rows it touches.  The exchange block
// for one destination is a RouteHeader, then up to route_cap RouteEntry in no
// particular order (workgroups append at atomically reserved offsets): the
// receiver keys its records by the draw id, so visibility sequences are the API
// order whatever order the entries arrive in.  A block that would hold more than
// route_cap entries keeps route_cap of them and says so (total > route_cap): its
// receiver then sets up every primitive of the draw itself (exact, slower).
struct alignas(16) RouteEntry {
    TriCompact rec;   // dx1 == kCompactLarge: a large primitive, whose setup the receiver re-runs
    uint32_t bb0, bb1;// clipped pixel bbox (BBox)
    uint32_t gid;     // draw primitive
    uint32_t pad;
};
static_assert(sizeof(RouteEntry) == 48, "RouteEntry must be 48 B");
struct alignas(16) RouteHeader {
    uint32_t pad0;
    uint32_t total;   // entries the sender had for this destination; the block holds min(total, route_cap)
    uint32_t pad[2];
};
static_assert(sizeof(RouteHeader) == 16, "RouteHeader must be 16 B");
__host__ __device__ inline uint64_t route_block_bytes(uint32_t cap) { return sizeof(RouteHeader) + (uint64_t)cap * sizeof(RouteEntry); }
#ifndef ZR_ROUTE_CHUNK
#define ZR_ROUTE_CHUNK 512
#endif
constexpr uint32_t kRouteChunk = ZR_ROUTE_CHUNK;
constexpr int kRouteThreads = ZR_ROUTE_CHUNK;   // 1 primitive per thread (a latency chain: index -> positions)
constexpr uint32_t kMaxShards = 32;  // destination masks are u32
// Scratch sets the runtime cycles through for overlapped draws: a partitioned
// draw's route + exchange, binning and tile pass are three pipeline stages on
// three streams, each stage of draw i + 2, i + 1 and i in a set of its own.
constexpr uint32_t kScratchSets = 3;

// Timing-experiment switches (ZR_DEBUG env var); never set in production runs.
enum : uint32_t { kDebugSkipRaster = 1u, kDebugSkipShade = 2u, kDebugLoadOnly = 16u,
                  kDebugPhase1Only = 32u, kDebugStamps = 128u,
                  kDebugReverseTiles = 256u, kDebugSkipLanePath = 512u, kDebugSkipWavePath = 1024u,
                  // timing only (ZR_TILE_DEBUG builds; wrong images): the resolve without one
                  // of its gathers -- vertex ids as 3t..3t+2, every attribute from vertex 0,
                  // every record from record 0 (docs/EXPERIMENTS.md, round 3)
                  kDebugIdentityVids = 2048u, kDebugSameVids = 4096u, kDebugSameRecord = 8192u };

// Status words in host-mapped pinned memory (read by the runtime at sync points).
constexpr uint32_t kSlabSlots = 48;  // draws per sync interval that report their slab target
enum StatusWord : uint32_t {
    kStTotalPairs = 0,      // (tile, primitive) pairs of the last draw (saturating)
    kStOverflow = 1,        // draws with a pair run the pool could not hold (since the last sync)
    // (word 2 unused)
    kStTrianglesSetup = 3,
    kStDroppedClip = 4,
    kStRouteMax = 5,        // partitioned draws: the largest per-destination entry total routed (since the last sync)
    kStRouteFallback = 6,   // partitioned draws whose received blocks overflowed (set up in full; since the last sync)
    kStMicro = 7,           // covered micro primitives of the last draw
    kStBinNeed = 8,         // the largest bin buffer a draw with a dropped run asked for since the last sync
                            // (entries, saturating): tiles x bin_slab_target + the pool entries its runs asked for
    kStPoolPairs = 9,       // pairs the last draw put in pool runs (saturating)
    kStPoolRuns = 10,       // pool runs of the last draw
    kStJobsDenied = 11,     // draws whose tile jobs did not fit DrawParams::job_pad / job_slots (since the last sync)
    kStJobs = 12,           // tile jobs of the last draw beyond one per tile
    kStSlabSlot0 = 16,      // [kSlabSlots]: the slab target (bin_slab_target) of the draw given slot i (DrawParams::stat_slot)
    kStPoolSlot0 = 64,      // [kSlabSlots]: the pool that draw's runs need (sub-pools x the fullest one's asks; saturating)
    kStMaxSlot0 = 112,      // [kSlabSlots]: that draw's longest tile list
    kStJobBufSlot0 = 160,   // [kSlabSlots]: the tile-job key buffers that draw's split tiles needed (0: no jobs built)
    kStJobPartSlot0 = 208,  // [kSlabSlots]: ... and the most parts (jobs past the first) it put on one XCD
    kStWords = 256,
};
// Device counters of k_setup_bin, read by the draw's k_tile (tile 0 reports them
// and resets them, as every tile resets its count, so a draw needs no memset).
enum CounterWord : uint32_t {
    kCtSetup = 0, kCtDropped = 1,
    kCtMaxTile = 2,   // the largest tile list of the draw (pairs, including any past the slab)
    kCtPairs = 4,     // u64 (words 4-5): (tile, primitive) pairs of the draw
    kCtSchedTicket = 6,  // k_setup_bin ticket groups past phase 2 (the last group's last workgroup builds the schedules)
    kCtMicro = 7,        // covered micro primitives of the draw (DrawParams::micro)
    kCtPoolRuns = 10,    // pool runs the draw registered
    kCtJobsDenied = 11,  // 1: the draw's tile jobs did not fit (build_job_schedule)
    kCtJobs = 12,        // tile jobs of the draw beyond one per tile
    kCtJobBufs = 13,     // key buffers the draw's split tiles needed (build_job_schedule; fitting or not)
    kCtJobXcdMax = 14,   // the most parts of the draw on one XCD (build_job_schedule)
    // Words each on a 64-B line of its own, kCtSpread apart (one returning atomic
    // per workgroup on a shared word queues the 256 workgroups on it at the memory
    // side: ~90 ns apiece, docs/EXPERIMENTS.md round 6):
    kCtPoolSub0 = 32,    // u64 x kPoolSubs: entries the runs of sub-pool k asked for (its bump allocator; may pass its size)
    kCtTicketGroup0 = kCtPoolSub0 + 16 * 16,  // x kTicketGroups: workgroups of ticket group g past phase 2
    kCtWords = kCtTicketGroup0 + 16 * 16,
};
constexpr uint32_t kCtSpread = 16;      // words between the spread counters (64 B)
constexpr uint32_t kPoolSubs = 16;      // pool regions, each the bump allocator of workgroups w % kPoolSubs
constexpr uint32_t kTicketGroup = 16;   // workgroups per ticket group (w / kTicketGroup)
static_assert(kMaxRunsPerTile / kTicketGroup <= 16u, "ticket-group words for the largest setup grid");
// draw_info words (written by k_setup_bin for k_tile)
enum DrawInfoWord : uint32_t {
    kInfoRecords = 0,     // setup records the overflow scan covers (bboxes[0, n))
    kInfoByPosition = 1,  // 1: bboxes are indexed by received position, records by gids[position] (records mode)
    kInfoJobEntries = 2,  // entries per tile job of the draw (0: one job per tile; k_setup_bin build_job_schedule)
    kInfoWords = 4,
};

struct DrawParams {
    // vertex input (binding 0) and index buffer
    const uint8_t* vb;
    uint64_t vb_bytes;
    const uint8_t* ib;
    uint64_t ib_bytes;
    uint64_t vid_count;       // vertex v has every attribute inside vb_bytes iff v < vid_count (host-computed)
    uint32_t ib_tris;         // u32 indices: triangle t's 3 indices lie inside ib_bytes iff t < ib_tris
    uint32_t stride;
    uint32_t nattr;
    uint32_t attr_offset[4];
    uint32_t attr_size[4];    // bytes of each input: 12 (R32G32B32_SFLOAT) or 8 (R32G32_SFLOAT)
    uint32_t index_size;      // 0 = non-indexed draw, 2 or 4
    uint32_t first;           // first_index / first_vertex
    int32_t vertex_offset;
    uint32_t tris_per_instance;
    uint32_t prims;           // tris_per_instance * instance_count
    // viewport transform (Vulkan 1.3 §Controlling the Viewport)
    float hw, hh, cx, cy, dr, dmin, dlo, dhi;
    // fragment rectangle = scissor ∩ render area ∩ attachment (inclusive)
    int32_t clip_x0, clip_y0, clip_x1, clip_y1;
    uint32_t cull_mode;
    int32_t front_face;
    // attachments
    uint32_t fb_w, fb_h;
    int32_t color_format;
    uint32_t color_bpp;       // 0 = no colour attachment
    uint8_t* color;
    float* depth;             // nullptr = no depth attachment
    uint32_t write_mask;
    int32_t ra_x0, ra_y0, ra_x1, ra_y1;  // render area ∩ attachment (inclusive)
    uint32_t clear_color_enable;
    uint32_t clear_color_packed;         // pre-encoded for 8-bit formats
    float clear_color[4];
    uint32_t clear_depth_enable;
    float clear_depth;
    uint32_t load_depth;      // initial depth from the attachment (LOAD)
    // depth test
    int32_t depth_mode;
    int32_t depth_op;         // VkCompareOp for the LastWins pre-test
    uint32_t depth_write_out; // write the winner's depth
    // shading
    int32_t program;
    uint32_t view_push;       // mesh program: the matrix is push[0, 16) instead of *view_proj (mesh_push.slang)
    const float* time_ptr;    // Time.time uniform (device) or nullptr
    const float* view_proj;   // mesh program: View.view_proj, 16 floats column-major (device)
    // tiling / sharding
    uint32_t tiles_x, tiles_y, shard_rank, shard_count, ntiles;
    // tile ownership of the shard (ShardGeom): round-robin rows [0, full_rows),
    // own_rows of them this rank's; of the leftover rows' tiles (row-major index i
    // from full_rows * tiles_x on) this rank owns [left_lo, left_hi)
    uint32_t full_rows, own_rows, left_lo, left_hi;
    uint32_t tile_threads;    // k_tile workgroup size: 256 or 512 (tile_threads_for)
    uint32_t rec_table;       // k_tile (512 threads): keep the record table for the resolve (use_record_table)
    // partitioned setup (records mode).  In records mode `prims` is
    // max(draw primitives, shard_count * route_cap); the setup pass runs over the
    // dense positions [0, sum of the blocks' counts) of the received entries and
    // stores each record at its draw id gids[j] (< draw_prims <= prims) -- or,
    // when a received block overflowed, sets up every draw primitive (gids[j] = j).
    uint32_t draw_prims;      // primitives of the draw (instances * triangles per instance)
    const uint8_t* rlist;     // received exchange blocks ([shard_count] x route_block_bytes(route_cap)), or nullptr
    uint32_t route_cap;       // entries per exchange block
    uint32_t* gids;           // records mode: the draw primitive at each dense position
    uint8_t* route_out;       // k_route: this rank's send blocks ([shard_count] x route_block_bytes(route_cap))
    uint32_t route_lo, route_hi, route_chunks;
    // scratch (binning without contended global atomics)
    TriCompact* records;      // [prims] compact records (every binned primitive)
    TriRecord* records_big;   // [prims] full records, written for large primitives only
    float4* mesh_edges;       // mesh program: [prims][3] homogeneous edge coefficients (shade_mesh)
    BBox* bboxes;             // [prims]; bb0 == kEmptyBox when culled / no owned tile
    uint32_t* tile_counts;    // [ntiles] pairs per tile | kCountRuns (zero between draws)
    uint32_t* draw_info;      // [kInfoWords] (DrawInfoWord)
    uint32_t* counters;       // [kCtWords] (CounterWord)
    uint32_t* bins;           // [pool_off + pool_cap] tile t's slab at [t * slab, (t + 1) * slab), then the pool
    uint32_t slab;            // slab entries per tile
    uint32_t setup_wgs;       // workgroups of k_setup_bin (one per CU at most)
    uint32_t unit_shift;      // log2 primitives per claim unit (64 lanes * batch * rounds)
    uint32_t units;           // claim units of the draw: ceil(prims / unit size)
    uint32_t setup_batch;     // primitives per lane in flight (template instance of k_setup_bin)
    uint32_t bbox_lds;        // 0: bboxes in global memory; else LDS entries per workgroup (own units * unit size)
    uint32_t bin_stage;       // k_setup_bin phase 4: LDS staging capacity in pairs (0: scatter straight to the bins)
    uint32_t debug;           // kDebug* bits (timing experiments only)
    unsigned long long* dbg_ts; // [setup_wgs][8] s_memrealtime stamps (kDebugStamps only)
    uint32_t* tile_order;     // tile schedule (k_setup_bin's last workgroup -> k_tile), or nullptr: xcd_tile order
    uint32_t* win_bits;       // winner census (zr_device_set_profiling level 2): bit p = draw primitive p won a pixel
    uint32_t* status;         // host-mapped
    // Micro primitives: k_setup_bin tests a primitive whose clipped
    // pixel bbox is a single pixel (a small one) for coverage of that pixel's
    // sample, and drops it -- no record, no bin entry -- when it yields no
    // fragment (C4: most of its 10M primitives).  0: off (ZR_MICRO=0, A/B).
    uint32_t micro;
    // Overflow runs: a workgroup whose run of pairs for tile t does
    // not fit what is left of t's slab stores it in the pool instead,
    // bins[pool_off + base, + its pairs) from a bump allocator (kCtPoolSub0, pool_commit), and
    // registers (pool_off + base, pairs) in runs[t * run_cap + w], w its
    // workgroup index (slots of other workgroups hold length 0).  The run that
    // straddles the slab end records its offset, the slab's fill (kRunFill); a run
    // the pool cannot hold is dropped (kRunDropped) and k_tile takes that tile by
    // its record scan.
    uint32_t pool_off, pool_cap, run_cap;
    uint32_t stat_slot;       // status slot for this draw's slab target (kStSlabSlot0 + i), or >= kSlabSlots: none
    uint2* runs;              // [ntiles * run_cap] (bins index, pairs), zero between draws (k_tile clears a used table)
    uint32_t* run_counts;     // [ntiles] run word (kRunFill, kRunDropped; zero between draws: k_tile resets it)
    // Tile jobs: a list longer than job_entries is split into
    // jobs of job_entries entries, each its own k_tile block (tile_order items
    // t | part << kJobTileBits, built by k_setup_bin's last workgroup), which
    // store their keys to job_keys[job_slot[t] + part]; the last job of the tile
    // (job_tickets) folds them in with a min and resolves it.  job_entries 0: off.
    // tile_order: [0, job_pad) parts 1.. (and spare kJobNone blocks), then the
    // tiles (the schedule, or xcd_tile order when tile_sched is 0).
    uint32_t job_entries, job_pad, job_slots;  // job_pad: k_tile blocks for parts 1.. (a multiple of 8)
    uint32_t tile_sched;             // 1: tile_order[job_pad, + ntiles) holds the heaviest-first tile schedule
    uint32_t* job_slot;              // [ntiles] first key buffer of a split tile (one per job)
    unsigned long long* job_keys;    // [job_slots][kTilePixels] key buffers
    uint32_t* job_tickets;           // [job_slots] per split tile, at its first buffer (zero between draws)
    // log2 of the draw's tile edge (kTileShiftMin..kTileShiftMax; tile_shift_for):
    // k_setup_bin bins and k_tile rasterizes tiles of 1 << tile_shift pixels a side
    uint32_t tile_shift;
    // push-constant state at the draw (zr_cmd_push_constants): the bytes ride in
    // the launch's kernel arguments, as Vulkan push constants ride in user SGPRs
    // (last, so the fields above keep their kernarg offsets; fields added later
    // go above it, after the older ones, for the same reason: k_tile's reloads of
    // the parameters are grouped scalar loads)
    float push[kMaxPushWords];
};

// k_tile workgroup size for a pass of `ntiles` tiles on `cus` CUs: 4 waves per
// tile while the pass has >= 6 tiles per CU, else 8 (tile-row shards: a tile's
// primitives spread over more waves).  Measured on C2 shards (1 GPU, rank 0 of
// G): G=4 tile pass 44 -> 39 us, G=8 40 -> 33 us; 16 waves per tile was slower
// than 4 (61 / 43 us), so it is not built.
// k_setup_bin LDS words besides the two tile arrays: misc (32) + list prefix (64)
// + the tile schedule's per-XCD bucket counts (8 x 64, the last workgroup only).
constexpr uint32_t kSchedBuckets = 64;
constexpr uint32_t kSetupMiscWords = 96 + 8 * kSchedBuckets;
// A draw of fewer than 32 primitives per tile (cerberus at 1080p: 16) also gets 8
// waves: its few heavy tiles (large triangles) end the pass alone on their CUs
// (cerberus tile pass 124 -> 113 us; C1, 49 per tile, is 14% slower at 8 waves).
// A draw of 80+ primitives per tile gets 8 waves too: its tiles are long enough
// for the extra waves to pay (round 1 v46, ZR_TILE_NT A/B: C2, 490 per tile,
// tile pass 78.9 -> 77.1 us; C4 equal.  Round 2, after the lane-walk changes:
// C3, 122 per tile, frame 250.7 -> 239.9 us at 8 waves; C1, 49 per tile, 54.5 ->
// 57.0 us, so it keeps 4).
// A partitioned shard whose 512-thread tile pass would take nearly every wave
// slot of the GPU (>= 3.5 tiles per CU) gets 4 waves per tile instead: the next
// draw's route, exchange and list setup on the setup stream then run beside the
// tile pass rather than after it (round 2, C3 rank 0 of 8 on one GPU: 67.5 ->
// 61.9 us per frame; replicated shards, whose single setup kernel needs whole
// CUs, are 13-20 % slower that way, and C2's shard of 8, at one tile per CU,
// equal).
// Round 4 (three-stage partitioned pipeline, balanced tile ownership): a
// partitioned shard whose tiles fit one round of 512-thread workgroups (4 per CU)
// takes 8 waves per tile -- C3 rank of 8 (1020 tiles), with the records-mode grid
// below: 4.47x vs 4.12x at 4 waves -- and 4 waves only past one round.
// 64-px tiles (4096 pixels, 32 KiB of keys) take 512 threads (4 workgroups per
// CU), or 1024 (2 per CU, LDS for the record table) for draws of at least one
// primitive per pixel -- round 6, 2 interleaved runs: C3 frame 230.2 us at 1024 vs
// 208.8 at 512 (tile pass 180.9 vs 156.3), C4 317.6 vs 322.1; 16-px tiles (256
// pixels) take 256.
inline uint32_t tile_threads_for(uint32_t ntiles, uint32_t cus, uint64_t prims, bool partitioned,
                                 uint32_t tile_shift = kTileShift) {
    if (tile_shift == 6u) return prims >= ((uint64_t)ntiles << 12) ? 1024u : 512u;
    if (tile_shift == 4u) return (uint32_t)kTileThreads;
    const uint32_t c = cus ? cus : 1u;
    const uint32_t per_cu = ntiles / c;
    if (partitioned) return ntiles > 4ull * c ? (uint32_t)kTileThreads : 512u;
    return (per_cu >= 6u && prims >= 32ull * ntiles && prims < 80ull * ntiles) ? (uint32_t)kTileThreads : 512u;
}

// k_setup_bin workgroups of a partitioned (records-mode) draw that expects about
// `entries` received records: one per 2048 entries (16 waves x 2 records per
// lane), at least 16, at most one per CU.  One per CU (the unpartitioned choice)
// left most of a workgroup's waves idle and multiplied the per-tile counter
// atomics (round 4, emulated rank of 8: C2 frame 43.6 -> 38.4 us, C3 equal).
// Whether k_setup_bin tests micro primitives for their one sample
// (DrawParams::micro): for draws of at least one primitive per pixel of the
// render area, whose mean primitive is then sub-pixel.  C4 (10M over 2.07M
// pixels): frame 406.9 -> 320.6 us; on C2 (0.5 per pixel, 0.15 % of its
// primitives micro) the test measured +1.7 us of setup for nothing, so sparser
// draws skip it (docs/EXPERIMENTS.md, round 5).
inline bool use_micro_test(uint64_t prims, uint64_t pixels) { return prims >= pixels; }

// The slab (entries per tile) a draw's tiles want: the draw's mean list length
// plus three standard deviations of a Poisson count plus 64, so uniform scenes do
// not overflow (C2: mean 645, longest 741, target 785) and skewed scenes put only
// their crowded tiles' excess in the pool.  Evaluated by k_tile's tile 0 (the
// draw's pair total is known there) and applied by the runtime to later draws.
__host__ __device__ inline uint32_t bin_slab_target(uint64_t pairs, uint32_t ntiles) {
    if (!ntiles) return 0;
    const float mean = (float)pairs / (float)ntiles;
    const float t = mean + 3.0f * sqrtf(mean) + 64.0f;
    return t >= (float)kMaxSlab ? kMaxSlab : (uint32_t)t;
}

// A slab of the longest list when that costs at most twice the target plus 1024
// entries per tile (the bin memory bound; 0 otherwise): a mildly
// skewed draw then keeps every list whole, no pool runs.  cerberus' ~80 runs a
// frame on its few crowded tiles -- the pass's critical path -- cost its tile
// pass ~1.8 us.
inline uint32_t bin_slab_whole(uint32_t target, uint32_t max_tile) {
    return (uint64_t)max_tile <= 2ull * target + 1024u ? max_tile : 0u;
}

// The bin buffer (entries) of a scratch set's first draw, before any draw has
// been measured: twice the primitives plus 256 per tile.  That draw takes slabs of
// a third of it (zr_runtime ensure_scratch) and the pool the rest, which holds
// the Gaussian-clustered c2x / c3x scenes' first frames without a dropped run.
constexpr uint32_t kBinShrinkSyncs = 16;  // the runtime's bin-buffer shrink check interval (sync points)
constexpr uint64_t kBinShrinkMin = 1ull << 24;  // ... and the least it frees (entries: 64 MiB)

inline uint64_t bin_default_capacity(uint64_t prims, uint32_t ntiles) {
    return std::max<uint64_t>(1ull << 20, 2 * prims + 256ull * ntiles);
}

// Tile jobs (DrawParams::job_entries): a shape whose longest list exceeded four
// jobs of kTileJobEntries (two 1024-entry segments each) splits its long lists
// -- one workgroup walking 30 segments of a crowded tile was the clustered c2x
// scene's tile pass.
constexpr uint32_t kTileJobEntries = 2048;
inline bool use_tile_jobs(uint32_t max_tile) { return max_tile > 4u * kTileJobEntries; }
// Key buffers a draw shape not measured yet may get for its tile jobs (64 MiB;
// zr_runtime ensure_scratch): afterwards a shape gets what its split needed.
constexpr uint64_t kJobKeyBytesFirst = 64ull << 20;

inline uint32_t records_setup_wgs(uint64_t entries, uint32_t cus) {
    const uint64_t w = (entries + 2047u) / 2048u;
    return (uint32_t)std::max<uint64_t>(1u, std::min<uint64_t>(cus ? cus : 1u, std::max<uint64_t>(16u, w)));
}

// Whether k_tile's 512-thread resolve reads its winners' records from the tile's
// LDS record table (zr_kernels.hip rec_table_insert): for draws of >= 256
// primitives per screen tile.  There most winners are distinct small primitives
// and the table saves one gather each (C2, 490 per tile: tile pass 72.4 -> 65.8
// us); with fewer, larger primitives per tile their pixels' record requests
// already merge and the inserts and lookups cost more than they save (C3, 122
// per tile: 174.6 -> 181.8 us).
// (Stated per pixel -- a quarter primitive per pixel -- so it carries over to
// other tile edges.)
inline bool use_record_table(uint64_t prims, uint32_t tiles_x, uint32_t tiles_y, uint32_t tile_shift = kTileShift) {
    return 4ull * prims >= ((uint64_t)tiles_x * tiles_y << (2u * tile_shift));
}

// Whether k_setup_bin builds a heaviest-first tile schedule for k_tile
// (build_tile_schedule): when the pass has more tiles than resident workgroup
// slots (4 per CU at 512 threads, 8 at 256), so that dispatch order decides which
// tiles end the pass, and the draw is sparse (< 32 primitives per tile), where a
// few heavy tiles (a real mesh's dense parts) otherwise end the pass alone.  On
// uniform soups the order gains nothing and the schedule costs setup its ticket
// (round 4, ZR_TILE_SCHED A/B, 2 runs: cerberus frame 53.8 -> 51.0 us; C2 108.4
// -> 113.7, C3 238.9 -> 245.0, C1 and C4 equal within 0.5 %).
inline bool use_tile_schedule(uint32_t ntiles, uint32_t cus, uint32_t tile_threads, uint64_t prims,
                              uint32_t tile_shift = kTileShift) {
    const uint64_t slots = (uint64_t)cus * (8u * kTileThreads / tile_threads);
    return ntiles > slots && 32ull * prims < ((uint64_t)ntiles << (2u * tile_shift));  // (< 1/32 primitive per pixel)
}

// Draw i+1's setup beside draw i's tile pass (zr_device_t::setup_overlap): small
// draws, tile-row shards, and draws of fewer primitives than pixels -- not a
// draw whose HBM-bound setup is the frame (C4's 4.8 per pixel: +28 % beside its
// tile pass; C2 -11 %, C3 -5 %, docs/EXPERIMENTS.md round 6).
inline bool use_overlap_setup(uint64_t prims, uint32_t w, uint32_t h, uint32_t shards) {
    return prims <= (1u << 18) || shards > 1 || prims < (uint64_t)w * h;
}

// A measured draw shape is crowded when its longest list needed tile jobs and is
// more than eight times its slab target (a skewed scene, not a dense uniform one:
// c2x 29.7k vs 785; C4's longest list is within 10 % of its mean).
inline bool crowded_shape(uint32_t max_tile, uint32_t target) {
    return use_tile_jobs(max_tile) && (uint64_t)max_tile > 8ull * target;
}

// k_tile instances exist for 16- and 64-px tiles only for these (program, depth
// mode) pairs (zr_kernels.hip launch_tile_pm); other draws keep 32-px tiles.
constexpr bool tile_variant_built(int program, int depth_mode) {
    return (program == kProgFlat || program == kProgBlinn) && depth_mode != kDepthLastWins;
}

// The tile edge of a draw (DrawParams::tile_shift), from the 16 / 32 / 64-px A/B of
// round 6 (docs/EXPERIMENTS.md; 2 interleaved runs, frame time):
//   - 64 px for a large target with a dense draw -- at least 4096 tiles of 32 px
//     and 64 primitives per such tile (C3, 1M at 4K: 239.9 -> 229.6 us, its setup
//     bins a quarter of the tiles: 59.3 -> 44.1 us, the tile pass equal) -- and for
//     draws of at least one primitive per pixel (C4: 321.8 -> 316.8 us);
//   - 16 px for a draw shape whose longest list needed tile jobs (a crowded
//     region: the clustered c2x, 219.1 -> 166.8 us, its crowded tiles' lists and
//     overdraw split four ways), when the target has at most kMaxTilesPerPass of
//     them;
//   - 32 px otherwise (C1 44.4 us vs 62.9 / 52.9 at 16 / 64, C2 108.9 vs 140.8 /
//     120.8, cerberus 34.5 vs 61.9 / 60.8), and always for tile-row shards, whose
//     ownership, row gather and exchange are in 32-px tiles (at 64 a C3 rank of 8
//     has one tile per CU: slowest rank 58.7-63.0 vs 54.7-58.9 us).
// `crowded`: the shape at the edge picked by size was measured and is skewed
// (crowded_shape).
inline uint32_t tile_shift_for(uint64_t prims, uint32_t width, uint32_t height, uint32_t shard_count, bool crowded) {
    if (shard_count > 1) return kTileShift;
    const uint64_t t32 = (uint64_t)((width + 31u) / 32u) * ((height + 31u) / 32u);
    const uint64_t t16 = (uint64_t)((width + 15u) / 16u) * ((height + 15u) / 16u);
    if (crowded) return t16 <= kMaxTilesPerPass ? 4u : kTileShift;
    if ((t32 >= 4096u && prims >= 64u * t32) || prims >= (uint64_t)width * height) return 6u;
    return kTileShift;
}

__host__ __device__ inline ShardGeom shard_geom(const DrawParams& P) {
    ShardGeom s;
    s.tiles_x = P.tiles_x;
    s.tiles_y = P.tiles_y;
    s.G = P.shard_count;
    s.rank = P.shard_rank;
    s.full_rows = P.full_rows;
    s.own_rows = P.own_rows;
    s.left_lo = P.left_lo;
    s.left_hi = P.left_hi;
    return s;
}

// Launchers (zr_kernels.hip).  All enqueue on `stream`; no host synchronisation.
void launch_setup_bin(const DrawParams& p, void* stream);  // setup + bin, one launch
size_t setup_bin_lds_bytes(uint32_t ntiles, uint32_t bbox_entries, uint32_t stage_pairs = 0);
const void* setup_bin_kernel(uint32_t batch, bool mesh);
void launch_tile(const DrawParams& p, void* stream);
void launch_clear(const DrawParams& p, void* stream);
void launch_route(const DrawParams& p, void* stream);


}  // namespace zr
