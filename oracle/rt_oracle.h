/*
 * rt_oracle.h — CPU ORACLE (test infrastructure, not product code).
 *
 * Scalar C restatement of the reference's ray-tracing path, used only by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, as the checker. Nothing in the
 * product (realtimeraytracing_gradproject_amd/) links or calls it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - OBJ ingest and camera lookAt: pinned against outputs of the reference's own C++ (glm
 *     harness in oracle/_ref, counts/first-vertex/first-face goldens recorded in SURVEY.md §8c).
 *   - HLSL shading, DXR traversal/intersection, DirectXMath inverse/normalize/SinCos: the reference
 *     runs only under D3D12/DXR on Windows, so these are parity unpinned against reference
 *     execution; they are restated from the source text (file:line cited per function in
 *     rt_oracle.c) and cross-checked by an independent numpy restatement (oracle/np_reference.py).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

typedef struct {
  uint32_t blas;
  float xform[12]; /* object-to-world 3x4 row-major */
  uint32_t instance_id;
  uint32_t hit_group; /* 0 model, 2 plane */
} oracle_instance;

typedef struct {
  float color[3];
  float position[3];
  float intensity;
} oracle_light;

/* ingest / host math */
int oracle_obj_parse(const char* text, size_t len, float** vtx6, uint32_t* nv, uint32_t** idx, uint32_t* ni);
void oracle_free(void* p);
int oracle_vertex_normals(float* vtx6, uint32_t nv, const uint32_t* idx, uint32_t ni);
void oracle_camera_lookat(const float eye[3], const float center[3], const float up[3], float view[16]);
void oracle_camera_buffer(const float view[16], uint32_t W, uint32_t H, float fov_deg, float znear, float zfar, float cb[64]);

/* scene */
oracle_scene* oracle_scene_create(void);
void oracle_scene_destroy(oracle_scene* s);
/* returns BLAS id >= 0, or < 0 on error. vtx6: {pos, normal} per vertex. idx NULL = non-indexed. */
int oracle_add_blas(oracle_scene* s, const float* vtx6, uint32_t nv, const uint32_t* idx, uint32_t icount);
int oracle_set_instances(oracle_scene* s, const oracle_instance* inst, uint32_t n);
/* info: out[0] prims, out[1] nodes, out[2] levels, out[3] worst-case traversal stack */
int oracle_blas_info(const oracle_scene* s, int blas, uint32_t out[4]);
int oracle_tlas_info(const oracle_scene* s, uint32_t out[4]);
int oracle_export_blas(const oracle_scene* s, int blas, void* nodes, void* tris);
int oracle_export_tlas(const oracle_scene* s, void* nodes);

/* render W x H (rows NULL = all). stats[12] accumulates (same slots as RT_STAT_*), may be NULL.
 * brute_force != 0: closest hit by testing every triangle of every instance (no BVH).
 * schedule: RT_SCHED_PACKET (0: 8 x 8 wave packets, as the device) or RT_SCHED_LANE (1: one
 * independent traversal per pixel). The image is the same; the traversal counters follow it. */
int oracle_render(const oracle_scene* s, const float cb[64], const oracle_light* lights, uint32_t nlights,
                  const float material[6], int mode, int spp, uint32_t W, uint32_t H, const uint32_t* rows,
                  uint32_t nrows, uint8_t* rgba8, float* rgba32f, int nthreads, uint64_t* stats,
                  int brute_force, int schedule);
/* the same, the packet schedule's tiles traced as the device's forced tile-balance layouts (rt_set_tile_balance
 * 2 / 3 / 4 -> split 1 / 2 / 3): every tile in 2 x 2 parts, in 4 x 4, or by position; each part one packet */
int oracle_render_split(const oracle_scene* s, const float cb[64], const oracle_light* lights, uint32_t nlights,
                        const float material[6], int mode, int spp, uint32_t W, uint32_t H, const uint32_t* rows,
                        uint32_t nrows, uint8_t* rgba8, float* rgba32f, int nthreads, uint64_t* stats,
                        int brute_force, int schedule, int split);
/* batch trace: rays n x 8 floats, ray_flags = D3D12_RAY_FLAG bits (0x04 first hit ends, 0x10 cull back
 * faces), hits n x 4 u32 (t bits, instance, prim, flag), uv n x 2 (may be NULL) */
void oracle_camera_rays(const float cb[64], uint32_t W, uint32_t H, const uint32_t* px, const uint32_t* py, uint32_t n,
                        float ox, float oy, float* rays);
int oracle_trace_rays(const oracle_scene* s, const float* rays, uint32_t n, uint32_t ray_flags, uint32_t* hits,
                      float* uv, int brute_force, uint64_t* stats);

/* raster fallback (rt_raster_draw), rt_raster_oracle.c: draws in order, each vtx6[d] with nvtx[d]
 * {pos, normal} vertices and ntri[d] triangles (idx[d] NULL = non-indexed). rgba8 W x H x 4;
 * depth_out (W x H floats) and prim_out (W x H, 0xffffffff = background) may be NULL. */
int oracle_raster(const float* const* vtx6, const uint32_t* nvtx, const uint32_t* const* idx, const uint32_t* ntri,
                  uint32_t ndraws, const float o2w3x4[12], const float cb[64], uint32_t W, uint32_t H,
                  uint8_t* rgba8, float* depth_out, uint32_t* prim_out);

/* shading building blocks exposed for known-answer tests */
void oracle_pbr(const float n[3], const float cam[3], const float P[3], const oracle_light* lights,
                uint32_t nlights, const float material[6], float out[3]);
void oracle_direct(const float n[3], const float P[3], const oracle_light* lights, uint32_t nlights,
                   const float albedo[3], float out[3]);
float oracle_pow(float x, float y);

#ifdef __cplusplus
}
#endif
#endif
