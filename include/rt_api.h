/*
 * rt_api.h — C-ABI drop-in boundary of the MI355X ray tracer.
 *
 * This is the boundary the reference's DXR path sits behind (D3D12 + nv_helpers_dx12).
 * Each entry point names the reference interface it replaces (file:line, relative to the
 * reference tree UtkuGokalp/RealTimeRayTracing_GradProject).
 *
 * Rules:
 *   - extern "C", plain pointers and sizes, no exceptions cross the boundary.
 *   - Non-zero rt_status == FAILED(hr) in the reference (ThrowIfFailed, DXSampleHelper.h:16-22).
 *     rt_last_error(ctx) returns the message of the last failure on that context.
 *   - Host inputs are copied during the call. Output device buffers are owned by the caller.
 *   - GPU work is stream-ordered on the hip_stream passed in (NULL = the context's stream),
 *     like command-list recording; synchronise with hipStreamSynchronize (== fence wait,
 *     D3D12HelloTriangle.cpp:627-647).
 *   - One context per host thread (the reference records on a single thread).
 *   - Functions in the "host services" section never touch the GPU: they run without one.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_API_VERSION 4

typedef struct rt_ctx* rt_ctx_t;
typedef struct rt_mesh* rt_mesh_t;
typedef uint32_t rt_blas_t;

typedef enum {
  RT_OK = 0,
  RT_E_INVALID = -1,     /* bad argument / misuse (reference: std::logic_error) */
  RT_E_OOM = -2,         /* device or host allocation failed */
  RT_E_HIP = -3,         /* a HIP runtime call failed (reference: FAILED(hr)) */
  RT_E_RCCL = -4,        /* a collective (RCCL) call failed: rt_comm_*, rt_render_strips */
  RT_E_UNSUPPORTED = -5, /* no gfx950 device / feature not built */
  RT_E_IO = -6           /* file could not be opened (reference: LoadObjFile returns false) */
} rt_status;

/* Hit groups, in the reference's SBT order (D3D12HelloTriangle.cpp:1064-1080). */
enum { RT_HITGROUP_MODEL = 0, RT_HITGROUP_SHADOW = 1, RT_HITGROUP_PLANE = 2 };

/* Shading modes of the trace kernel. */
enum {
  RT_SHADE_REF = 0,            /* exact reference: ClosestHit (Lambert+PBR over the lights) for models,
                                  PlaneClosestHit (light 0 + one shadow ray) for the plane, Miss sky
                                  (Hit.hlsl:183-241, Miss.hlsl:3-10, ShadowRay.hlsl:10-20) */
  RT_SHADE_LAMBERT_SHADOW = 1, /* perf configs: every hit, one shadow ray per light */
  RT_SHADE_PRIMARY = 2         /* primary rays only: Lambert over the lights, no shadow rays (config C1) */
};

/* Trace schedules of the one-launch frame kernel (raygen + traversal + shading + shadow rays).
 * Same image; the traversal counters (rt_stats) follow the schedule. */
enum {
  RT_SCHED_PACKET = 0, /* default: each wave (8 x 8 pixels) walks the trees as one packet: scalar
                          node fetches, ballot child decisions, a wave-uniform stack. Runs when the
                          scene's worst-case stack is below 64 entries, else falls back to LANE */
  RT_SCHED_LANE = 1    /* one independent traversal per lane (LDS stack + HBM overflow) */
};

/* One TLAS instance (TopLevelASGenerator::AddInstance, TopLevelASGenerator.h:88-99,
 * instance desc fill TopLevelASGenerator.cpp:180-198). xform = object-to-world 3x4, row-major,
 * column-vector convention: world = M * (x,y,z,1). instance_id = InstanceID() (the list index in
 * the reference, D3D12HelloTriangle.cpp:749). */
typedef struct {
  rt_blas_t blas;
  float xform3x4_rowmajor[12];
  uint32_t instance_id;
  uint32_t hit_group; /* RT_HITGROUP_MODEL or RT_HITGROUP_PLANE */
} rt_instance;

/* == Hit.hlsl Light (Hit.hlsl:25-30) */
typedef struct {
  float color[3];
  float position[3];
  float intensity;
} rt_light;

/* == Hit.hlsl Material (Hit.hlsl:10-16), 24 B */
typedef struct {
  float albedo[3];
  float roughness, metallic, reflectivity;
} rt_material;

/* BVH summary returned by rt_blas_info / rt_tlas_info. */
typedef struct {
  uint32_t prim_count;   /* triangles (BLAS) or instances (TLAS) */
  uint32_t node_count;   /* 4-wide nodes (BFS order, root 0) */
  uint32_t depth;        /* levels of 4-wide nodes */
  uint32_t max_stack;    /* worst-case traversal-stack entries a path through this tree needs */
  float bounds_lo[3];
  float bounds_hi[3];
  double build_ms;       /* device time of the last build (HIP events) */
} rt_bvh_info;

/* Counters reported by rt_stats (accumulated over dispatches launched while stats are on). */
enum {
  RT_STAT_PRIMARY_RAYS = 0,
  RT_STAT_SHADOW_RAYS = 1,
  RT_STAT_AABB_TESTS = 2,  /* child-box slab tests (one per valid child of a visited node) */
  RT_STAT_TRI_TESTS = 3,   /* Moller-Trumbore tests */
  RT_STAT_INSTANCE_ENTRIES = 4,
  RT_STAT_STACK_OVERFLOWS = 5,
  RT_STAT_PIXELS = 6,
  RT_STAT_DISPATCHES = 7,
  RT_STAT_REFLECTION_RAYS = 8, /* RT_SHADE_REF with reflectivity != 0 (Hit.hlsl:176-203) */
  /* Fetches, the roofline's byte counts: in the packet schedule once per WAVE per visit (the node,
   * triangle or instance record is loaded once into SGPRs for the whole packet), in the per-lane
   * schedule once per lane per visit. */
  RT_STAT_NODE_FETCHES = 9,     /* 128-B BVH4 node records */
  RT_STAT_TRI_FETCHES = 10,     /* 48-B triangle records */
  RT_STAT_INSTANCE_FETCHES = 11, /* instance-record loads on a TLAS -> BLAS hand-off */
  RT_STAT_COUNT = 12
};

/* ------------------------------------------------------------------------------------------ */
/* Context                                                                                     */
/* ------------------------------------------------------------------------------------------ */

/* Replaces device/queue creation in D3D12HelloTriangle::LoadPipeline (D3D12HelloTriangle.cpp:85-198)
 * and CheckRaytracingSupport (:649). Fails with RT_E_UNSUPPORTED unless the device is gfx950. */
rt_status rt_create(int hip_device, rt_ctx_t* out);
/* Replaces OnDestroy + ComPtr release (D3D12HelloTriangle.cpp OnDestroy). */
rt_status rt_destroy(rt_ctx_t ctx);
const char* rt_last_error(rt_ctx_t ctx);
const char* rt_status_string(rt_status st);
int rt_api_version(void);

/* ------------------------------------------------------------------------------------------ */
/* Acceleration structures                                                                     */
/* ------------------------------------------------------------------------------------------ */

/* Replaces BottomLevelASGenerator::AddVertexBuffer + ComputeASBufferSizes + Generate
 * (BottomLevelASGenerator.h:106-153, .cpp:74-245; call site D3D12HelloTriangle.cpp:682-732).
 * vtx: host array, vcount vertices of `stride` bytes with float3 position at offset 0 and, when
 * stride >= 24, float3 normal at offset 12 (the reference Vertex, D3D12HelloTriangle.h:51-56).
 * idx: host uint32 triangle list (icount % 3 == 0) or NULL for non-indexed geometry
 * (vcount % 3 == 0). Builds an LBVH on the device (Morton codes, LDS radix sort, Karras
 * hierarchy, bottom-up refit). Synchronous: returns after the build has completed. */
rt_status rt_blas_build(rt_ctx_t ctx, const void* vtx, uint32_t vcount, uint32_t stride,
                        const uint32_t* idx, uint32_t icount, rt_blas_t* out);
/* Model hot-reload (D3D12HelloTriangle.cpp:1482-1596): rebuild an existing BLAS in place with new
 * geometry. Instances that reference it pick it up at the next rt_tlas_build. */
rt_status rt_blas_rebuild(rt_ctx_t ctx, rt_blas_t blas, const void* vtx, uint32_t vcount,
                          uint32_t stride, const uint32_t* idx, uint32_t icount);
rt_status rt_blas_info(rt_ctx_t ctx, rt_blas_t blas, rt_bvh_info* out);
/* Copies the BLAS to host memory for parity checks: nodes (node_count x 128 B 4-wide nodes, BFS order),
 * tris (prim_count x 48 B: v0.xyz,prim | e1.xyz,0 | e2.xyz,0 in leaf order). Either may be NULL. */
rt_status rt_blas_export(rt_ctx_t ctx, rt_blas_t blas, void* nodes, size_t nodes_bytes, void* tris,
                         size_t tris_bytes);

/* Replaces TopLevelASGenerator::AddInstance + ComputeASBufferSizes + Generate
 * (TopLevelASGenerator.h:88-130, .cpp:64-249; call site D3D12HelloTriangle.cpp:734-776), and
 * UpdateInstancePropertiesBuffer (D3D12HelloTriangle.cpp:1181-1204): the per-instance normal
 * matrix transpose(inverse(upper3x3)) is derived here. update_only != 0 refits the existing TLAS
 * (same instance count and BLAS ids; new transforms), as TopLevelASGenerator.cpp:202-222.
 * Double-buffered: launches already issued keep reading the previous version while this one is built into
 * the other (a per-frame update with frames in flight); the build waits on the device for the launches of
 * the version it overwrites, launches issued after it wait for it on the device, and the host returns once
 * this build's own kernels finished (the tree's size and stack bound come back). Only a changed layout (a
 * BLAS built or rebuilt since, or more instances than ever before) waits for all in-flight work. */
rt_status rt_tlas_build(rt_ctx_t ctx, const rt_instance* instances, uint32_t n, int update_only);
rt_status rt_tlas_info(rt_ctx_t ctx, rt_bvh_info* out);
/* Host wall time of the last rt_tlas_build call (ms), beside rt_bvh_info.build_ms (its kernels' device time). */
double rt_tlas_build_wall_ms(rt_ctx_t ctx);
/* nodes: node_count x 128 B 4-wide nodes; leaf refs are ~instance_index. */
rt_status rt_tlas_export(rt_ctx_t ctx, void* nodes, size_t nodes_bytes);

/* ------------------------------------------------------------------------------------------ */
/* Per-frame state                                                                             */
/* ------------------------------------------------------------------------------------------ */

/* Replaces UpdateCameraBuffer (D3D12HelloTriangle.cpp:1144-1170): cb = view, proj, viewInv,
 * projInv, 4 x 16 floats, each in XMMATRIX memory order (the exact 256-B constant buffer). */
rt_status rt_set_camera(rt_ctx_t ctx, const float cb[64]);
/* Replaces the Hit.hlsl light table (Hit.hlsl:48-57) and UpdateMaterialsBuffer/OnUpdate
 * (D3D12HelloTriangle.cpp:424-428). nlights in [1, 16]. spp in {1, 4, 9, 16} (k x k stratified). */
rt_status rt_set_shading(rt_ctx_t ctx, const rt_light* lights, uint32_t nlights,
                         const rt_material* material, int shade_mode, int spp);
/* RT_SCHED_PACKET (default) or RT_SCHED_LANE. */
rt_status rt_set_schedule(rt_ctx_t ctx, int schedule);
/* Packet schedule, one-sample frames: rows of the 8-pixel-wide tile one wave traces — 8 (default: 8 x 8, every
 * lane a pixel) or 4 (8 x 4, half the lanes idle). Same image either way. 4 makes the waves shorter: it pays
 * only when few enough waves run that the slowest tile sets the frame time, as in one rank's strips of a
 * frame tiled over many GPUs (C4 over 8 ranks: 0.196 -> 0.135 ms); otherwise it halves throughput. No reference
 * counterpart (DispatchRays schedules rays itself). */
rt_status rt_set_tile_rows(rt_ctx_t ctx, int rows);
/* Tile balance of the packet schedule (no reference counterpart: DispatchRays schedules rays itself). A wave walks
 * the union of its 8 x 8 tile's ray paths, so a frame lasts as long as its slowest tiles (on C4 one tile takes as
 * long as the rest of the frame). mode 1 (default, adaptive): every wave records its tile's time; when the last
 * frame of the same shape (size, row list, frames per launch) had tiles far above the mean, a one-workgroup plan
 * kernel before the launch splits the tiles above max(load bound, the finest split's floor) into 4, 16 or 64 sub-packets and
 * deals every wave longest first. The image never depends on it. 0: off (the plain grid). 2 / 3 / 4 / 5 (tests):
 * every tile in 4 parts / in 16 parts / by position (tx + 2 ty) % 3 whole, 4, 16 / in 64 one-pixel parts — also
 * under rt_set_stats, so the counters can be compared with the oracle's emulation of the same parts. A launch
 * whose forced layout would exceed 32768 waves (all its frames) fails with RT_E_UNSUPPORTED and renders nothing;
 * the adaptive mode has no such limit. */
rt_status rt_set_tile_balance(rt_ctx_t ctx, int mode);
/* The last launch shape's tile balance: out[0] plans run, [1] tiles split by the last plan, [2] its work items,
 * [3] the extra-wave budget, [4] the costliest / [5] the mean tile time (10-ns ticks), [6] the split threshold,
 * [7] launches of the shape, [8] the last plan found the costliest tile above the load bound (its list is not the
 * plain order), [9] tiles the lists failed to cover exactly once, [10] the first such tile, [11] its check word
 * ([9..11] only when the context was created with RT_BALANCE_CHECK=1 in the environment: a cover check after each
 * plan, diagnostics), [12..14] the last plan kernel's phases in 10-ns ticks (snapshot + load bound, budget,
 * placement), [15] the wave slots of the last plan's load bound (the list kernel's occupancy per CU, from the
 * runtime, x CUs), [16] work items the plans refused for want of budget (summed; a plan that refuses any item falls
 * back to the plain grid's list, so no part is ever dropped), [17] the plans that fell back, [18..19] 0. Host-side
 * read of host-mapped memory (may lag the device by a few launches). */
#define RT_BALANCE_INFO_COUNT 20
/* rt_tile_balance_info_n fills min(n, RT_BALANCE_INFO_COUNT) words of out (the array may grow in later versions:
 * pass its capacity). rt_tile_balance_info is the round-4 entry point and fills exactly its 16 words ([0..15]). */
rt_status rt_tile_balance_info_n(rt_ctx_t ctx, uint32_t* out, uint32_t n);
#define RT_BALANCE_INFO_COUNT_V1 16
rt_status rt_tile_balance_info(rt_ctx_t ctx, uint32_t out[RT_BALANCE_INFO_COUNT_V1]);
/* Context diagnostics: out[0] device-wide synchronisations so far (builds, rebuilds, buffer growth: never a frame
 * launch on a steady pipeline), [1] tile-balance maps recycled for a new launch shape (only once every stream that
 * used them is idle and none of them was used in the last 64 shape lookups: host queries, no synchronisation), [2]
 * launches that ran the plain grid because no map was free (after a miss the table is rescanned only every 16 such
 * launches), [3] maps held, [4] recycled maps that went on to start a plan (recycling that paid off).
 * rt_ctx_counters_n fills min(n, RT_CTX_COUNTERS_V2) words; rt_ctx_counters exactly its 4 ([0..3]). */
#define RT_CTX_COUNTERS 4
#define RT_CTX_COUNTERS_V2 5
rt_status rt_ctx_counters_n(rt_ctx_t ctx, uint64_t* out, uint32_t n);
rt_status rt_ctx_counters(rt_ctx_t ctx, uint64_t out[RT_CTX_COUNTERS]);
/* Enables device counters (rt_stats). Costs time: off for timed runs. */
rt_status rt_set_stats(rt_ctx_t ctx, int enable);

/* ------------------------------------------------------------------------------------------ */
/* Launch                                                                                      */
/* ------------------------------------------------------------------------------------------ */

/* Replaces DispatchRays (D3D12HelloTriangle.cpp:558-592) + RayGen/Hit/Miss/ShadowRay programs.
 * Renders an image of W x H. rows: host list of global row indices to render (NULL = all H
 * rows, in order); the output is compact: row r of the output is global row rows[r].
 * rgba8_dev: device buffer of nrows*W*4 bytes, R8G8B8A8_UNORM (D3D12HelloTriangle.cpp:971).
 * rgba32f_dev: optional device buffer of nrows*W*4 floats (the pre-quantisation float4), or NULL.
 * hip_stream: hipStream_t or NULL (context stream). Asynchronous, and frames may be in flight on several
 * streams at once (the reference keeps two frames in its swap chain): the per-launch device scratch — the row
 * list's device copy and, for trees deeper than the 32-entry LDS stack, the HBM overflow stack — comes from a
 * small ring of slots, each ordered on the device after the other streams' last uses of it (no host wait). */
rt_status rt_dispatch_rays(rt_ctx_t ctx, uint32_t W, uint32_t H, const uint32_t* rows,
                           uint32_t nrows, void* rgba8_dev, float* rgba32f_dev, void* hip_stream);
/* nframes (1 .. 4) full W x H frames in ONE launch (the grid's z): frame z with the 64-float camera buffer
 * cameras[64 z ..] (NULL: the context's camera for every frame, which rt_set_camera must then have set), written as
 * R8G8B8A8_UNORM at rgba8_dev + z * frame_stride bytes (0: W * H * 4, the frames back to back; else at least one
 * frame and a multiple of 4: RT_E_INVALID otherwise). Each frame equals the one
 * rt_dispatch_rays renders with that camera. No reference counterpart (one DispatchRays per frame,
 * D3D12HelloTriangle.cpp:584-592): a batch of views or of consecutive frames pays one launch and one host issue,
 * and the frames' waves share one grid (no tail between them). Same stream rules as rt_dispatch_rays. */
rt_status rt_dispatch_frames(rt_ctx_t ctx, uint32_t W, uint32_t H, uint32_t nframes, const float* cameras,
                             void* rgba8_dev, uint64_t frame_stride, void* hip_stream);
/* Stream lifetime: the context notes (host-side, no event per launch) which streams launched with the current
 * TLAS version, and records one event on each of them when the next rt_tlas_build swaps that version out; the tile
 * balance likewise notes the streams that read a work list, and queries the stream of a shape's previous launch
 * (whether frames are in flight). A caller that destroys a stream it launched on (rt_dispatch_rays,
 * rt_trace_rays) calls rt_forget_stream(ctx, stream) first: the events are recorded now, while the stream is valid,
 * and the context holds no handle to it afterwards. (The reference's command lists and fences have no equivalent:
 * D3D12HelloTriangle.cpp:627-647 waits for the GPU every frame.) */
rt_status rt_forget_stream(rt_ctx_t ctx, void* hip_stream);

/* TraceRay ray flags (the D3D12_RAY_FLAG values the reference passes, Common.hlsl:44-82). */
enum {
  RT_RAY_FLAG_NONE = 0x00,
  RT_RAY_FLAG_ACCEPT_FIRST_HIT_AND_END_SEARCH = 0x04, /* any hit: first accepted hit ends the ray */
  RT_RAY_FLAG_CULL_BACK_FACING_TRIANGLES = 0x10,      /* CastReflectionRay (Common.hlsl:58-69) */
  RT_RAY_FLAG_CULL_FRONT_FACING_TRIANGLES = 0x20      /* DXR flag; not set by the reference's shaders */
};

/* Batch TraceRay (Common.hlsl:44-82 semantics) for parity tests and external callers.
 * rays_dev: n x 8 floats (o.x,o.y,o.z,tmin, d.x,d.y,d.z,tmax), direction used as given.
 * ray_flags: RT_RAY_FLAG_* (other bits, or both cull flags: RT_E_INVALID). Front faces are clockwise seen from the
 * ray origin (DXR's default), flipped by an instance transform with a negative determinant.
 * hits_dev: n x 4 x 32-bit: (t as float, instance_id, primitive index, hit flag) with u,v written
 * to uv_dev (n x 2 floats) when uv_dev != NULL. A miss has hit flag 0 and t = tmax. Asynchronous; may run
 * concurrently with frames and other batches on other streams (per-launch overflow stack, as rt_dispatch_rays). */
rt_status rt_trace_rays(rt_ctx_t ctx, const float* rays_dev, uint32_t n, uint32_t ray_flags,
                        uint32_t* hits_dev, float* uv_dev, void* hip_stream);

/* Raster fallback: the reference's abandoned rasterization pipeline (shaders/shaders.hlsl:41-59,
 * recorded at D3D12HelloTriangle.cpp:513-540, pipeline state :248-276). Draws the BLAS vertex
 * buffers `draws[0..ndraws)` in order (indexed when built with indices; the reference draws the
 * model, then the plane) through VSMain: pos = projection * view * objectToWorld * (p, 1), with
 * view = cb[0..15] and projection = cb[16..31] of rt_set_camera and objectToWorld the 3x4
 * row-major transform given (the reference binds instance 0's; NULL = identity). D3D rules:
 * clip 0 <= z <= w, 16.8 fixed-point snap, pixel centres, top-left fill rule, back faces culled
 * (clockwise = front), depth LESS on a D32 buffer cleared to 1.0. PSMain returns the interpolated
 * COLOR (the reference's input layout: the 16 bytes at offset 12 of each vertex = normal.xyz +
 * next vertex's position.x; 0 for the last vertex). rgba8: W x H RGBA8 (cleared to
 * {0.03, 0.35, 0.43, 1}); depth32f: optional W x H floats. Device pointers, on `stream`.
 * Asynchronous, except the first draw of a context (one 4-byte read-back sizes the tile bins) and
 * draws that must grow buffers or upload a changed draw list (they wait for in-flight work). The raster
 * scratch is per context: a draw issued on another stream than the previous draw waits for it on the device.
 * Test hook: the environment variable RT_RASTER_BIN_CAP caps the tile-bin capacity (a draw that
 * overflows it renders the same image through the slower slot walk). */
rt_status rt_raster_draw(rt_ctx_t ctx, const rt_blas_t* draws, uint32_t ndraws, const float* object_to_world,
                         uint32_t W, uint32_t H, void* rgba8, float* depth32f, void* stream);

/* Multi-GPU frame assembly: un-interleaves `nranks` compact strip images gathered back to back in
 * `gathered_dev` (rank-major; rank k holds strips s with s % nranks == k, strip_rows rows each)
 * into a full W x H RGBA8 image. Asynchronous. */
rt_status rt_assemble_strips(rt_ctx_t ctx, uint32_t W, uint32_t H, uint32_t nranks,
                             uint32_t strip_rows, const void* gathered_dev, void* rgba8_dev,
                             void* hip_stream);
/* Host helper: the row list rank `rank` of `nranks` renders with interleaved strips of
 * strip_rows rows. Writes up to cap rows to rows_out; returns the row count (0 on bad args). */
uint32_t rt_strip_rows(uint32_t H, uint32_t nranks, uint32_t rank, uint32_t strip_rows,
                       uint32_t* rows_out, uint32_t cap);
/* Frame-pipeline events for the strips loop (render of frame k + 1 beside the gather + assembly of
 * frame k on a second stream). No reference counterpart (the reference renders on one GPU): plain
 * hipEvent_t handles without timestamps and without the system-scope fence hipEventRecord performs
 * by default (both streams are on one device; the consumer is a kernel, not the host), which takes
 * ~3 us off every record on the frame's critical path. rt_stream_wait_event(stream, ev) makes
 * later work on `stream` wait for the last record of `ev`. */
rt_status rt_event_create(void** ev_out);
rt_status rt_event_destroy(void* ev);
rt_status rt_event_record(void* ev, void* hip_stream);
rt_status rt_stream_wait_event(void* hip_stream, void* ev);

/* ---- Multi-GPU frame loop ---------------------------------------------------------
 * One frame (the reference's DispatchRays W x H, D3D12HelloTriangle.cpp:584-592) tiled over N ranks, one
 * process and one rt_ctx per GPU, each holding the full scene: rank r renders the interleaved strips
 * s % N == r (strip_rows rows each) into a compact buffer, one ncclGather (rccl.h:745) brings every rank's
 * buffer to rank 0, and rt_assemble_strips un-interleaves them there. No reference counterpart (the reference
 * renders on one GPU). RCCL is loaded at run time (librccl.so.1; RT_E_UNSUPPORTED when absent). */
typedef struct rt_comm* rt_comm_t;
#define RT_COMM_ID_BYTES 128 /* == sizeof(ncclUniqueId) */
/* RT_OK when RCCL can be loaded (no collective, no GPU work): callers decide on the tiled-frame loop before
 * the collective rt_comm_init. */
rt_status rt_comm_available(void);
/* ncclGetUniqueId: rank 0 creates the id; the caller hands the 128 bytes to every rank (MPI, a file, a
 * torch.distributed broadcast). */
rt_status rt_comm_get_unique_id(void* id_out);
/* ncclCommInitRank on the context's device. Collective: returns once all nranks ranks have joined. */
rt_status rt_comm_init(rt_ctx_t ctx, uint32_t nranks, uint32_t rank, const void* id, rt_comm_t* out);
/* Test transport, no RCCL: ONE process stands in for all `nranks` ranks on the context's GPU (1 .. 64). Each
 * rt_render_strips renders every rank's strips into that rank's block of the pipeline slot, and the gather is a
 * device copy into rank 0's rank-major buffer, issued on the gather stream by the issue thread at the point where
 * the RCCL communicator calls ncclGather. Strip plan, frame batching, events, tails and the rank-strided assembly
 * are the RCCL path's, so the N > 1 frame layout runs on a one-GPU box. The communicator is rank 0. */
rt_status rt_comm_init_loopback(rt_ctx_t ctx, uint32_t nranks, rt_comm_t* out);
/* Loopback rehearsal of one rank's share of the cost (tools/share_ceiling.py): from the next frame on, only the
 * emulated ranks [first, first + count) render; the others' blocks of the slot keep whatever they hold, while the
 * gather copy and rank 0's assembly still move and assemble every rank's block. A step then costs this process what
 * it costs rank `first` of an N-rank run (its strips' render, the gather, the assembly), minus the xGMI transfer;
 * the frames hold stale strips for the ranks not rendered. count 0: every rank (the default). Loopback
 * communicators only (RT_E_INVALID otherwise). No reference counterpart. */
rt_status rt_comm_loopback_render_ranks(rt_comm_t comm, uint32_t first, uint32_t count);
/* Drains the pipeline first (a partly filled slot is gathered and assembled as it is, every rank alike: destroy
 * is collective like the frames), then stops the issue thread. Destroy communicators before their context. */
rt_status rt_comm_destroy(rt_comm_t comm);
/* The failure path (SURVEY.md §5 "Failure detection"; the reference's only failure handling is ThrowIfFailed,
 * DXSampleHelper.h:16-22): frees the communicator WITHOUT issuing another collective, so one rank can leave on an
 * error while the others may never call again. The partly filled slot is discarded (never gathered or assembled),
 * steps not yet handed to the issue thread are dropped, the issue thread stops, and ncclCommAbort cancels the
 * collectives in flight (their peers may never match them). Local, unlike rt_comm_destroy. The frames of discarded or
 * cancelled steps have undefined content; the context stays usable. Destroy communicators before their context. */
rt_status rt_comm_abort(rt_comm_t comm);
const char* rt_comm_last_error(rt_comm_t comm);
/* The communicator's gather stream, made to wait (on the device) for every step issued so far, the
 * assemblies on the render streams included: work the caller enqueues on it after this call sees rank 0's
 * frames complete. */
void* rt_comm_stream(rt_comm_t comm);
rt_status rt_comm_synchronize(rt_comm_t comm);
/* Pipeline slots (= the communicator's render streams, frames in flight with render_stream NULL): one per
 * hardware queue beside the gather stream's (GPU_MAX_HW_QUEUES - 1, HIP's default 4 gives 3; RT_COMM_SLOTS
 * overrides, 1..8). Call k uses slot k mod depth. */
uint32_t rt_comm_pipeline_depth(rt_comm_t comm);

/* Frames per gather (1 .. 4; default 1): consecutive rt_render_strips calls render into one pipeline slot and ONE
 * ncclGather moves all their strips, so the gather half of a step (a stream wait, the RCCL call, an event) is paid
 * once per `frames_per_gather` frames; the bytes moved per frame are the same. A frame's assembly then waits for the
 * last frame of its slot (or for rt_comm_stream / rt_comm_synchronize, which gather a partly filled slot as it is).
 * Every rank must set the same value between the same two calls (it changes the collective's size). Drains the
 * pipeline. rt_comm_pipeline_depth becomes slots x frames_per_gather. Replaces: nothing in the reference (the
 * multi-GPU loop is this library's). */
rt_status rt_comm_set_batch(rt_comm_t comm, uint32_t frames_per_gather);
uint32_t rt_comm_batch(rt_comm_t comm);
/* Phase timing of the loop on this rank (diagnostics for the multi-GPU bench line; no reference counterpart — the
 * reference has no multi-GPU path, its frame spans submit -> fence, D3D12HelloTriangle.cpp:436-470). When on, each
 * step records timing-event pairs around its render launches (render stream; every emulated rank's on a loopback), its gather (gather stream: from the
 * moment this rank's render is done to the gather's end, any wait for the other ranks inside the collective
 * included) and rank 0's assembly, and the host time of each rt_render_strips* call and of the issue thread's work.
 * Drains the pipeline (like rt_comm_set_batch: every rank between the same calls) and resets the sums. */
rt_status rt_comm_set_phase_timing(rt_comm_t comm, int on);
/* The sums since rt_comm_set_phase_timing(on) (drains the pipeline first). out[0] frames, [1] render launches, [2]
 * their summed ms, [3] gathers, [4] summed ms, [5] assemblies (rank 0), [6] summed ms, [7] caller host us summed over
 * [8] calls, [9] the issue thread's host us, [10] bytes into rank 0 from the other ranks, [11] bytes of every rank's
 * block. Fills min(n, RT_COMM_PHASE_COUNT) doubles. */
#define RT_COMM_PHASE_COUNT 12
rt_status rt_comm_phase_stats(rt_comm_t comm, double* out, uint32_t n);
/* One tiled frame, collective over the ranks (every rank calls it, in the same frame order): this rank's
 * strips are rendered on render_stream into one of the communicator's pipeline slots (NULL: slot k's own
 * stream of the communicator; its render streams and its gather stream sit on separate hardware queues). The
 * strips are RGB8 (3 bytes a pixel: the alpha byte of the frame is the constant 255 and is restored by the
 * assembly, so it never crosses xGMI). The gather stream waits for that render (a device-side event) and runs ONE
 * ncclGather of every rank's slot into rank 0; the step's tail returns to render_stream: a wait for that gather
 * and, on rank 0, the assembly of the W x H RGBA8 frame into frame_out (device buffer; ignored on other ranks).
 * The tail is issued by a later call once the gather is enqueued, at the latest before the slot renders again (or
 * by rt_comm_stream / rt_comm_synchronize). The slot's next render on the same stream follows its tail in stream
 * order; a slot moved to another stream, and two assemblies into one frame_out on different streams, are ordered
 * by events. With rt_comm_set_batch(b > 1) a slot's later frames may name another render_stream than its first:
 * the slot's stream then waits for the work already queued on that stream before rendering the frame, and the
 * frame's tail is returned to it by an event. No host waits: frame k's gather overlaps frame k + 1's render, and
 * frames on different streams overlap (frames in flight). Asynchronous: frame_out is complete once the work
 * enqueued on rt_comm_stream(comm) after that call has run, or after rt_comm_synchronize. Streams passed must
 * stay valid until then. */
rt_status rt_render_strips(rt_comm_t comm, uint32_t W, uint32_t H, uint32_t strip_rows, void* frame_out,
                           void* render_stream);
/* nframes (1 .. rt_comm_batch, at most 4) consecutive frames of the loop in ONE call: this rank renders their
 * strips in ONE launch (the frame index is the launch's third grid dimension, so a rank's share of several frames
 * fills the GPU as one grid and pays one launch) into one pipeline slot; frame b uses the camera buffer
 * cameras[64 b .. 64 b + 63] (rt_set_camera's layout; NULL: the context's camera for every frame) and is assembled
 * on rank 0 into frames_out[b]. Frames that do not fit the slot being filled start a new slot. Otherwise exactly
 * nframes calls of rt_render_strips (lights, material, TLAS are the context's at the call). */
rt_status rt_render_strips_frames(rt_comm_t comm, uint32_t W, uint32_t H, uint32_t strip_rows, uint32_t nframes,
                                  const float* cameras, void* const* frames_out, void* render_stream);

/* Copies the counters (RT_STAT_*) to out[RT_STAT_COUNT]; synchronises the context. */
rt_status rt_stats(rt_ctx_t ctx, uint64_t out[RT_STAT_COUNT]);
rt_status rt_stats_reset(rt_ctx_t ctx);

/* ------------------------------------------------------------------------------------------ */
/* Host services (no GPU): mesh ingest, normals, plane, camera                                 */
/* ------------------------------------------------------------------------------------------ */

/* OBJFileManager::LoadObjFile (OBJ_FileManager.cpp:10-71): `v x y z` and `f i j k` lines only,
 * 1-based -> 0-based unsigned indices. RT_E_IO if the file cannot be opened. */
rt_status rt_mesh_load_obj(const char* path, rt_mesh_t* out);
/* Same parser over an in-memory text buffer. */
rt_status rt_mesh_parse_obj(const char* text, size_t len, rt_mesh_t* out);
void rt_mesh_free(rt_mesh_t mesh);
uint32_t rt_mesh_vertex_count(rt_mesh_t mesh);
uint32_t rt_mesh_index_count(rt_mesh_t mesh);
/* Vertex array, 6 floats per vertex {pos.xyz, normal.xyz} (reference Vertex, stride 24). Normals
 * are the default (0,1,0) until rt_mesh_compute_vertex_normals. */
const float* rt_mesh_vertices(rt_mesh_t mesh);
const uint32_t* rt_mesh_indices(rt_mesh_t mesh);
/* D3D12HelloTriangle::ComputeVertexNormals (D3D12HelloTriangle.cpp:1430-1462). */
rt_status rt_mesh_compute_vertex_normals(rt_mesh_t mesh);

/* CreatePlaneVB (D3D12HelloTriangle.cpp:1237-1271): 6 vertices x {pos, normal} = 36 floats. */
void rt_plane_vertices(float out[36]);

/* Manipulator::setLookat + update (manipulator.cpp:26-32, 305-314) == glm::lookAtRH
 * (glm/gtc/matrix_transform.inl:519-545): view matrix in glm column-major memory order. */
void rt_camera_lookat(const float eye[3], const float center[3], const float up[3], float view[16]);
/* UpdateCameraBuffer (D3D12HelloTriangle.cpp:1144-1170): cb = {view (as given), proj =
 * XMMatrixPerspectiveFovRH(fov_deg, W/H, znear, zfar), inverse(view), inverse(proj)}. */
void rt_camera_buffer(const float view[16], uint32_t W, uint32_t H, float fov_deg, float znear,
                      float zfar, float cb[64]);

/* ---- Camera manipulator ------------------------------------------------------------------------
 * nv_helpers_dx12::Manipulator (include/manipulator.h:33-148, src/manipulator.cpp) as plain data the
 * caller owns, so any FFI can hold it; every function is host-only arithmetic (no GPU). Float
 * results are bit-identical to the reference's glm 0.9.8.5 arithmetic (tests/golden/manipulator.json).
 * `mode` and `speed` are written directly (Manipulator::setMode / setSpeed, :50-53, :91-94);
 * `matrix` is what getMatrix returns (:83-86), column-major as glm stores it. */
typedef enum rt_manip_mode {  /* Manipulator::Modes, manipulator.h:37 */
  RT_MANIP_EXAMINE = 0,
  RT_MANIP_FLY = 1,
  RT_MANIP_WALK = 2,
  RT_MANIP_TRACKBALL = 3
} rt_manip_mode;

typedef enum rt_manip_action {  /* Manipulator::Actions, manipulator.h:38 */
  RT_MANIP_NONE = 0,
  RT_MANIP_ORBIT = 1,
  RT_MANIP_DOLLY = 2,
  RT_MANIP_PAN = 3,
  RT_MANIP_LOOK_AROUND = 4
} rt_manip_action;

/* Manipulator::Inputs (manipulator.h:39-40) as a bit set. */
#define RT_INPUT_LMB 0x01u
#define RT_INPUT_MMB 0x02u
#define RT_INPUT_RMB 0x04u
#define RT_INPUT_SHIFT 0x08u
#define RT_INPUT_CTRL 0x10u
#define RT_INPUT_ALT 0x20u

typedef struct rt_manipulator {  /* member defaults: manipulator.h:124-144 */
  float pos[3];      /* m_pos  (10,10,10) */
  float interest[3]; /* m_int  (0,0,0) */
  float up[3];       /* m_up   (0,1,0) */
  float roll;        /* m_roll radians about the view z axis */
  float matrix[16];  /* m_matrix */
  int32_t width;     /* m_width  1 */
  int32_t height;    /* m_height 1 */
  float speed;       /* m_speed  30 */
  float mouse[2];    /* m_mouse */
  float tbsize;      /* m_tbsize 0.8 */
  int32_t mode;      /* rt_manip_mode */
} rt_manipulator;    /* 132 bytes */

/* Manipulator::Manipulator (:17-20): member defaults, then update(). */
void rt_manip_init(rt_manipulator* m);
/* Manipulator::update (:305-314): matrix = lookAt(pos, interest, up) [* rotate(roll, z)]. */
void rt_manip_update(rt_manipulator* m);
/* setLookat (:26-32), setRoll (:66-70), setWindowSize (:125-129), setMousePosition (:107-111). */
void rt_manip_set_lookat(rt_manipulator* m, const float eye[3], const float center[3], const float up[3]);
void rt_manip_set_roll(rt_manipulator* m, float roll);
void rt_manip_set_window_size(rt_manipulator* m, int32_t w, int32_t h);
void rt_manip_set_mouse_position(rt_manipulator* m, int32_t x, int32_t y);
/* motion (:135-166): apply `action` for a mouse move to (x, y), update, remember (x, y). */
void rt_manip_motion(rt_manipulator* m, int32_t x, int32_t y, int32_t action);
/* mouseMove (:175-198): choose the action from the RT_INPUT_* bits, apply it; returns the action. */
int32_t rt_manip_mouse_move(rt_manipulator* m, int32_t x, int32_t y, uint32_t inputs);
/* wheel (:203-214): dolly by value*|value|/width*speed, then update. */
void rt_manip_wheel(rt_manipulator* m, int32_t value);

#ifdef __cplusplus
}
#endif

#endif /* RT_API_H */
