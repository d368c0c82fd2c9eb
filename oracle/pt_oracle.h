/*
 * pt_oracle.h — CPU restatement of the reference path tracer's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker: it is
 * loaded by tests/, by __graft_entry__.smoke() and by bench.py's
 * cpu_baseline leg, and by nothing else.  The product (libpt.so) never
 * links, loads or calls it.
 *
 * Parity status: pinned statistically against the reference's committed
 * render output2/exp2.png (TRIANGLEWORLD, see tests/golden/); the LBVH
 * topology, closest-hit and scatter restatements follow the reference
 * source line by line (citations in pt_oracle.cpp).  The reference itself
 * cannot be built here (needs nvcc + cuRAND + GLFW), so
 * bit-level parity against a reference binary is unpinned.
 *
 * All structs are plain C, binary-identical to include/pt.h's.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_SPHERE = 1, ORC_TRIANGLE = 3 };            /* simulation/cuda_object.h:12-14 */
enum { ORC_LAMBERTIAN = 1, ORC_METAL = 2, ORC_DIELECTRIC = 4 }; /* simulation/material.h:13-15 */

typedef struct { int32_t type; int32_t mat; float v[9]; } orc_object;          /* sphere: c[3], r | tri: v0,v1,v2 */
typedef struct { int32_t type; float albedo[3]; float fuzz; float ir; } orc_material;
typedef struct {
    float origin[3], lower_left[3], horizontal[3], vertical[3];
    float right[3], up[3], front[3];
    float focus_dist, lens_radius, time0, time1;
} orc_camera;
typedef struct { int32_t left, right, parent, objid; float bmin[3], bmax[3]; } orc_node;   /* utils/bvh_node.h:8-17 */
typedef struct { int32_t hit, obj, mat, front_face; float t, p[3], n[3]; } orc_hit;
typedef struct { uint64_t rays, node_visits, box_tests, tri_tests, sphere_tests, paths; } orc_stats;

/* camera.h:12-39 (host ctor) */
void orc_camera_make(const float from[3], const float at[3], float vfov, float aspect,
                     float aperture, float focus, float t0, float t1, orc_camera* out);

/* cuRAND XORWOW semantics: curand_init(seed, subsequence, 0) (main.cu:268) */
void orc_xorwow_init(uint64_t seed, uint64_t subsequence, uint32_t state[6]);  /* d, v0..v4 */
void orc_xorwow_init_range(uint64_t seed, uint64_t first, int64_t count, uint32_t* states);
void orc_xorwow_skip_subsequences(uint32_t state[6], uint64_t n);   /* state := state after n*2^67 draws */
uint32_t orc_xorwow_next(uint32_t state[6]);
float orc_curand_uniform(uint32_t state[6]);
/* test-only: 1 = the three draws of vec3(u-0.5f, u-0.5f, u-0.5f) taken z, y, x (an unpinned choice, see draw3) */
void orc_set_draw_order(int zyx);

/* utils/morton_code.h:29-75; include_origin=1 reproduces maxBox starting as the zero box */
int orc_morton_keys(const orc_object* objs, int64_t n, int include_origin, uint64_t* keys_out);
/* utils/bvh.h:71-130; tight=1 grows internal boxes from their children only,
 * tight=0 reproduces the reference's origin-seeded boxes (bvh.h:124-127). */
int orc_build_lbvh(const orc_object* objs, int64_t n, const uint64_t* keys, int tight, orc_node* nodes);
int orc_bvh_depth(const orc_node* nodes, int64_t n);

/* utils/render_manager.h:71-135: closest hit, t in [tmin, tmax).  rays: n x {o[3], d[3]} */
int orc_trace(const orc_object* objs, int64_t nobj, const orc_node* nodes, const float* rays,
              int64_t nrays, float tmin, float tmax, int brute, orc_hit* hits, orc_stats* stats);

/* simulation/material.h:28-61 driven by a tape of uniforms; returns scatter() */
int orc_scatter_tape(const orc_material* m, const float ray[6], const orc_hit* rec,
                     const float* tape, int tape_len, int* used, float out_ray[6], float atten[3]);

/* main.cu:271-294 over the rows listed in `rows` (global row indices, row 0 = bottom).
 * states: one XORWOW state per pixel of the listed rows (row-major, in `rows` order), updated.
 * out_rgb: same pixel order, 3 floats each, sqrt-gamma applied (main.cu:290-293). */
int orc_render(const orc_object* objs, int64_t nobj, const orc_material* mats, int64_t nmat,
               const orc_node* nodes, const orc_camera* cam, int width, int height,
               const int32_t* rows, int nrows, int spp, int max_depth,
               uint32_t* states, float* out_rgb, orc_stats* stats, int nthreads);

/* orc_render plus per-pixel ray counts (diagnostics). */
int orc_render2(const orc_object* objs, int64_t nobj, const orc_material* mats, int64_t nmat,
                const orc_node* nodes, const orc_camera* cam, int width, int height,
                const int32_t* rows, int nrows, int spp, int max_depth,
                uint32_t* states, float* out_rgb, orc_stats* stats, int nthreads, uint32_t* pixel_rays);

/* Sample mode: pixel-sample (p, s) draws from a XORWOW state seeded by one Philox4x32-10
 * block (key = seed, counter = {s, p_lo, p_hi, "SAMP"}); samples summed per chunk of `chunk`
 * samples, chunk sums summed in order, sqrt(total / spp).  Same rows/out layout as orc_render. */
int orc_render_sample(const orc_object* objs, int64_t nobj, const orc_material* mats, int64_t nmat,
                      const orc_node* nodes, const orc_camera* cam, int width, int height,
                      const int32_t* rows, int nrows, int spp, int max_depth, uint64_t seed, int chunk,
                      float* out_rgb, orc_stats* stats, int nthreads);

/* orc_render2 that also writes the raw per-pixel sample sums (before sqrt(sum / spp)) to
 * out_sum (3 floats per pixel) when non-null: the input of progressive accumulation. */
int orc_render3(const orc_object* objs, int64_t nobj, const orc_material* mats, int64_t nmat,
                const orc_node* nodes, const orc_camera* cam, int width, int height,
                const int32_t* rows, int nrows, int spp, int max_depth,
                uint32_t* states, float* out_rgb, orc_stats* stats, int nthreads, uint32_t* pixel_rays,
                float* out_sum);

/* orc_render_sample whose samples are numbered from sample_base (a progressive frame continues
 * the sample sequence), plus the raw per-pixel sums (chunk sums added in order) when out_sum. */
int orc_render_sample2(const orc_object* objs, int64_t nobj, const orc_material* mats, int64_t nmat,
                       const orc_node* nodes, const orc_camera* cam, int width, int height,
                       const int32_t* rows, int nrows, int spp, int max_depth, uint64_t seed, int chunk,
                       float* out_rgb, orc_stats* stats, int nthreads, uint32_t sample_base, float* out_sum);
uint32_t orc_philox_word(uint64_t key, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, int word);
void orc_sample_stream(uint64_t seed, uint32_t sample, uint64_t pixel, uint32_t state[6]);  /* {d, v0..v4} */

#ifdef __cplusplus
}
#endif
#endif
