/*
 * pt.h — C ABI of the MI355X-native path tracer (libpt.so).
 *
 * The reference (Nablax/Path-Tracer-CUDA-OpenGL) has no plugin/FFI layer: its boundary is
 * the set of CUDA kernel launches and host helpers in main.cu / utils/bvh.h.  Each entry
 * point below names the reference interface it replaces.  All functions return PT_OK (0)
 * or a PT_ERR_* code; the message of the last failure on the calling thread is returned by
 * pt_last_error().  No torch or HIP types appear in any signature: device pointers and
 * streams are passed as plain pointers.
 *
 * Threading: one pt_scene / pt_film per device; calls on different objects may come from
 * different threads.  There is no global mutable state besides the thread-local error.
 */
#ifndef PT_H
#define PT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 1

enum pt_status {
    PT_OK = 0,
    PT_ERR_INVALID = 1,   /* bad argument */
    PT_ERR_HIP = 2,       /* HIP runtime error (reference: checkCudaErrors, cuda_check.h:8-17) */
    PT_ERR_IO = 3,        /* file could not be read / written */
    PT_ERR_NOMEM = 4,
    PT_ERR_NODEVICE = 5,  /* no GPU visible: the library never falls back to the CPU */
    PT_ERR_STATE = 6      /* e.g. render before the BVH was built */
};

/* Object and material types: simulation/cuda_object.h:12-14, simulation/material.h:13-15 */
enum { PT_SPHERE = 1, PT_TRIANGLE = 3 };
enum { PT_LAMBERTIAN = 1, PT_METAL = 2, PT_DIELECTRIC = 4 };

/* One scene object, the reference's CudaObj (cuda_object.h:16-123) without device pointers.
 * sphere: v[0..2] = centre, v[3] = radius (negative radius = hollow sphere, as in RTIOW)
 * triangle: v[0..2], v[3..5], v[6..8] = vertices v0, v1, v2 (one CudaObj per triangle). */
typedef struct { int32_t type; int32_t mat; float v[9]; } pt_object;

/* Material (material.h:17-68) in its constructed state: fuzz already clamped to <= 1. */
typedef struct { int32_t type; float albedo[3]; float fuzz; float ir; } pt_material;

/* camera (camera.h:10-76) after its host constructor ran (see pt_camera_make). */
typedef struct {
    float origin[3], lower_left[3], horizontal[3], vertical[3];
    float right[3], up[3], front[3];
    float focus_dist, lens_radius, time0, time1;
} pt_camera;

typedef struct { float o[3]; float d[3]; } pt_ray;                       /* simulation/ray.h */
typedef struct { int32_t hit, obj, mat, front_face; float t, p[3], n[3]; } pt_hit; /* hit_record.h:12-25 */
/* BVH node in the reference's layout (utils/bvh_node.h:8-17): internal nodes [0, n-2], root 0,
 * leaves [n-1, 2n-2]; objid = -1 for internal nodes. */
typedef struct { int32_t left, right, parent, objid; float bmin[3], bmax[3]; } pt_bvh_node;

/* Work counters of one pt_render / pt_trace_closest call (counted in-kernel). */
typedef struct {
    uint64_t rays;          /* closest-hit queries: primary + every bounce */
    uint64_t node_visits;   /* internal BVH nodes popped (each = 2 child-box tests) */
    uint64_t box_tests;
    uint64_t tri_tests;
    uint64_t sphere_tests;
    uint64_t paths;         /* camera samples */
    double kernel_ms;       /* device time of the render/trace kernel(s), HIP events */
    uint64_t algo_bytes;    /* 56*node_visits + 40*tri_tests + 20*sphere_tests */
} pt_stats;

/* A complete host-side scene description (objects, materials, camera, frame settings). */
typedef struct {
    pt_object* objects; int64_t n_objects;
    pt_material* materials; int64_t n_materials;
    pt_camera camera;
    int32_t width, height, spp, max_depth;
    char name[64];
} pt_scene_desc;

/* Instancing.  An instance places mesh `mesh` (a range of objects, in object
 * space) in the world by the affine transform world = m * (object, 1), m row-major 3 x 4. */
typedef struct { float m[12]; int32_t mesh; int32_t reserved; } pt_instance;
/* An instanced scene description (pt_preset_instanced): meshes = object ranges
 * [mesh_first[i], mesh_first[i] + mesh_count[i]) of `objects`. */
typedef struct {
    pt_object* objects; int64_t n_objects;
    int64_t* mesh_first; int64_t* mesh_count; int32_t n_meshes;
    pt_instance* instances; int64_t n_instances;
    pt_material* materials; int64_t n_materials;
    pt_camera camera;
    int32_t width, height, spp, max_depth;
    char name[64];
} pt_instanced_desc;

typedef struct pt_scene pt_scene;   /* device-resident objects, materials, LBVH */
typedef struct pt_film pt_film;     /* device-resident per-pixel RNG streams for a set of rows */

const char* pt_last_error(void);
int pt_abi_version(void);
int pt_device_count(int* count);

/* ---------------------------------------------------------------- host-side surface (no GPU) */
/* camera host ctor, camera.h:12-39 */
int pt_camera_make(const float from[3], const float at[3], float vfov_deg, float aspect,
                   float aperture, float focus_dist, float time0, float time1, pt_camera* out);
/* camera::processKeyboard, camera.h:41-56 (dir: 0 FORWARD 1 BACKWARD 2 LEFT 3 RIGHT 4 UP 5 DOWN) */
int pt_camera_move(pt_camera* cam, int dir, float delta_time);
/* Scene builders.  name: "triangle_world" (main.cu:119-196, the reference default),
 * "random_world" (main.cu:198-256), "test_world" (main.cu:57-117), "rtiow" (C1),
 * "cornell" (C2), "bunny_cornell" (C3), "bunny_field" (C5), "bunny_field_x4" (C5 at 4x the
 * triangles: 840 half-size bunnies, an HBM-resident stress case).  models_dir holds
 * cornellbox/<part>.obj and bunny/bunny.obj.  width/height <= 0 keep the preset's frame. */
int pt_preset_scene(const char* name, const char* models_dir, int width, int height, pt_scene_desc* out);
void pt_scene_desc_free(pt_scene_desc* desc);
/* The instanced form of a preset: "bunny_field" (C5: the Cornell box once and the bunny mesh,
 * scaled x250 in object space, placed 210 times by translations -- the same grid, order and frame
 * as pt_preset_scene's flattened 1,043,312 triangles), "bunny_cornell" (box + one bunny), "cornell"
 * (the box alone).  The box is instance 0 with the identity transform. */
int pt_preset_instanced(const char* name, const char* models_dir, int width, int height, pt_instanced_desc* out);
void pt_instanced_desc_free(pt_instanced_desc* desc);
/* OBJ mesh -> triangle objects (objl::Loader::LoadFile, OBJ_Loader.hpp:426-708, flattened to
 * one pt_object per triangle); v' = v * scale + translate.  *out is freed with pt_free. */
int pt_load_obj(const char* path, float scale, const float translate[3], int32_t mat,
                pt_object** out, int64_t* count);
void pt_free(void* p);
/* Morton keys (code << 32 | objID), stable-sorted by code: morton::computeMortonOnHost,
 * morton_code.h:64-75.  include_origin=1 seeds the scene box with the zero box (main.cu:122). */
int pt_morton_keys(const pt_object* objs, int64_t n, int include_origin, uint64_t* keys);
/* PngImage::saveColor + write (png_image.h:24-37; main.cu:477-484): rgb is row-major with
 * row 0 = bottom (as the render kernel writes it); rows are flipped on output. */
int pt_write_png(const char* path, const float* rgb, int width, int height);
/* Quantise exactly like saveColor: (uint8)(clamp(c, 0, 0.999) * 256), alpha 255, row flip. */
int pt_quantize_rgba8(const float* rgb, int width, int height, uint8_t* rgba);
/* PngImage::write of an already quantised frame (pt_render_ex with PT_OUT_RGBA8): rgba is
 * row-major with row 0 = bottom, flipped on output like pt_write_png. */
int pt_write_png_rgba8(const char* path, const uint8_t* rgba, int width, int height);

/* ---------------------------------------------------------------- device (MI355X, gfx950) */
/* Replaces the scene upload of generate*WorldOnHost (main.cu:173-192: cudaMalloc/cudaMemcpy,
 * copyObjMatsToDevice, one copyTrianglesToDevice<<<1,1>>> per triangle). */
int pt_scene_create(int device, const pt_object* objs, int64_t n_objects,
                    const pt_material* mats, int64_t n_materials, pt_scene** out);
/* Replaces lbvh::buildBVH (bvh.h:132-145), entirely on the device: scene box, Morton codes
 * (morton_code.h:19-45), a stable radix sort by code (the reference's host std::stable_sort,
 * morton_code.h:64-75), leaf records, Karras hierarchy (bvh.h:17-115), bottom-up refit with
 * tight internal boxes (growBBox, bvh.h:117-130).  flags: PT_BVH_ORIGIN_BOUNDS (default
 * behaviour of the reference: the Morton bounds contain the origin, main.cu:122);
 * PT_BVH_HOST_KEYS computes and sorts the keys on the host instead (identical result; A/B). */
#define PT_BVH_ORIGIN_BOUNDS 1
#define PT_BVH_HOST_KEYS 2
/* PT_BVH_WIDE_DEVICE: also build the wide kernel's compressed 8-wide tree, on the device, in the
 * same call (top-down SAH + collapse, a few milliseconds even at a million primitives; for
 * dynamic scenes rebuilt every frame).  Without it PT_KERNEL_WIDE builds the tree at first use on
 * the host (binned SAH, slower to build; PT_WIDE_BUILD=device selects the device build there
 * too; after pt_scene_update_objects the device build is the default).  Either tree gives the
 * same images. */
#define PT_BVH_WIDE_DEVICE 4
int pt_scene_build_bvh(pt_scene* scene, int flags);
/* pt_scene_build_bvh with its device work enqueued on `stream` (a hipStream_t, NULL = the null
 * stream) instead of the null stream; returns when the build is complete (the tree depth is read
 * back to pick the traversal kernel). */
int pt_scene_build_bvh_ex(pt_scene* scene, int flags, void* stream);
/* An instanced scene (the reference has none: its MeshLoader is a stub,
 * mesh_loader.h:9-16, and every triangle is its own object with its own cudaMalloc, main.cu:182-190).
 * Each mesh is stored once, in object space; pt_scene_build_bvh builds a two-level tree: one
 * bottom-level 8-wide tree per mesh and a top-level tree over the instances' world boxes, all in
 * one node array.  Rays enter an instance transformed by the inverse of its matrix (the hit's t is
 * the same parameter in both spaces); normals return by the inverse transpose.  Renders and traces
 * use the wide kernel only (PT_KERNEL_WIDE or PT_KERNEL_DEFAULT).  Because the ray is transformed,
 * results equal the flattened scene's within floating-point tolerance (tests/test_gpu_instancing.py
 * states it), not bit for bit; ties between equal t are decided by (instance, primitive).  Hit
 * records report obj = the object's index in the flattened order (instances in order, each
 * contributing its mesh's objects). */
int pt_scene_create_instanced(int device, const pt_object* objs, int64_t n_objects, const int64_t* mesh_first,
                              const int64_t* mesh_count, int n_meshes, const pt_instance* instances, int64_t n_instances,
                              const pt_material* mats, int64_t n_materials, pt_scene** out);
/* Dynamic scenes (per-frame rebuild): overwrite objects [first, first + n)
 * (host array; same validation as pt_scene_create) and mark the hierarchy stale -- rendering or
 * tracing fails with PT_ERR_STATE until pt_scene_build_bvh runs again.  A rebuild reuses every
 * device buffer of the previous build (no allocation, no device-wide synchronisation).  The
 * reference has no counterpart: it builds once (main.cu:122-128 / bvh.h:132-145). */
int pt_scene_update_objects(pt_scene* scene, const pt_object* objs, int64_t first, int64_t n);
/* Device time of the last pt_scene_build_bvh (HIP events around the build's stream work). */
int pt_scene_build_time(pt_scene* scene, double* ms);
int pt_scene_bvh_info(pt_scene* scene, int* depth, int64_t* n_nodes, int64_t* device_bytes);
/* The wide tree of the current build (0s before its first use): depth (levels), node slots,
 * build time in ms (wall time of the host build + upload, or of the device build when built at
 * first use; 0 when pt_scene_build_bvh built it -- then it is in pt_scene_build_time), source
 * (0 none, 1 host SAH, 2 device SAH or PLOC). */
int pt_scene_wide_info(pt_scene* scene, int* depth, int64_t* node_slots, double* build_ms, int* source);
/* Download the LBVH in the reference's node layout (2n-1 nodes). */
int pt_scene_download_bvh(pt_scene* scene, pt_bvh_node* nodes);
/* RenderManager::hitBvh (render_manager.h:86-135) over a batch of rays, t in [tmin, tmax).
 * rays/hits are host pointers. */
int pt_trace_closest(pt_scene* scene, const pt_ray* rays, int64_t n, float tmin, float tmax,
                     pt_hit* hits, pt_stats* stats);
/* pt_trace_closest with a choice of tree: PT_KERNEL_WIDE traverses the compressed 8-wide tree
 * (see pt_render_ex); any other value the binary LBVH in the reference's order.  Same hits. */
int pt_trace_closest_ex(pt_scene* scene, const pt_ray* rays, int64_t n, float tmin, float tmax, int kernel,
                        pt_hit* hits, pt_stats* stats);
/* pt_trace_closest_ex on device-resident arrays (e.g. torch tensors): rays / hits are device
 * pointers, traced on `stream` (a hipStream_t, may be NULL); returns when the batch is done. */
int pt_trace_closest_device(pt_scene* scene, const pt_ray* rays, int64_t n, float tmin, float tmax, int kernel,
                            pt_hit* hits, void* stream, pt_stats* stats);
/* Per-pixel XORWOW streams, initRandom (main.cu:262-269): curand_init(seed, pixel, 0, ...)
 * for every pixel of the rows this film owns.  Rows are grouped in stripes of stripe_height;
 * stripe s belongs to part (s % n_parts).  n_parts = 1 owns the whole frame. */
int pt_film_create(int device, int width, int height, int stripe_height, int n_parts, int part,
                   uint64_t seed, pt_film** out);
int pt_film_info(pt_film* film, int* n_rows, int64_t* n_pixels);
int pt_film_rows(pt_film* film, int32_t* rows);                  /* global row of each local row */
int pt_film_get_rng(pt_film* film, uint32_t* states);            /* n_pixels x {d, v0..v4} */
int pt_film_set_rng(pt_film* film, const uint32_t* states);
/* render<<<>>> (main.cu:271-294): spp samples per pixel of the film's rows, max_depth bounces.
 * Writes sqrt(mean) RGB, 3 floats per pixel, local rows in order.  out_rgb is a device
 * pointer when out_on_device != 0 (then `stream` is the hipStream_t to use, may be NULL),
 * else a host pointer.  The film's RNG streams advance, as the reference's devStates do.
 * Asynchronous when out_on_device != 0 and stats == NULL: the call enqueues the frame's kernels
 * (render, resolve, the next launch's tile order) on `stream` and returns without waiting for the
 * device; pt_film_stats() then gives the frame's counters.  With stats != NULL, or a host output,
 * the call returns when the frame is done.  Frames of one film must use one stream (or be ordered
 * by the caller): the film's buffers are reused by the next frame. */
int pt_render(pt_scene* scene, pt_film* film, const pt_camera* cam, int spp, int max_depth,
              float* out_rgb, int out_on_device, void* stream, pt_stats* stats);
/* Render options.
 * kernel: PT_KERNEL_DEFAULT (= PT_KERNEL_WIDE unless the PT_RENDER_KERNEL environment
 *   variable says "simple" or "wavefront"), PT_KERNEL_SIMPLE (ray-synchronous, the reference's loop
 *   structure, binary LBVH), PT_KERNEL_WAVEFRONT (per-lane state machine, steps chosen by wave
 *   ballots, binary LBVH, the reference's visiting order) or PT_KERNEL_WIDE (the same state
 *   machine on a compressed 8-wide SAH tree built on the host at first use, nearest child first;
 *   the closest hit is chosen by (t, the reference's tie order), so the hits are the reference's).
 *   All kernels give bit-identical images for a given rng mode.
 * rng: PT_RNG_COMPAT (default): the reference's semantics -- one cuRAND-XORWOW stream per
 *   pixel, curand_init(seed, pixel, 0), samples consumed in order and kept across calls like
 *   the reference's devStates; a pixel's samples are inherently sequential.
 *   PT_RNG_SAMPLE: one XORWOW stream per pixel-sample (the reference's generator and
 *   curand_uniform mapping), its state seeded by one Philox4x32-10 block with key = film seed and
 *   counter = {sample, pixel, 0, "SAMP"}; samples are summed in blocks of `chunk` samples
 *   (0 = max(16, ceil(spp/64))), each block's fp32 sum is converted to 32.32 fixed point and the
 *   pixel's blocks are added exactly (integer atomics: the order in which blocks finish does not
 *   matter).  (pixel, block) tasks are handed to persistent waves, longest tiles first from the
 *   previous launch's costs; neither the scheduling nor the stripe partition changes the image.
 *   Deterministic, statistically identical to the reference, not its random numbers; does not
 *   advance the film's XORWOW streams.  Needs 32 bytes of device memory per pixel
 *   ({x, y, z, rays} accumulators), whatever the spp.
 *   The wide kernel builds its tree on the host at the first render after each
 *   pt_scene_build_bvh (C3 5,000 triangles ~5 ms, C5 1.04 M ~0.8 s) unless the build was asked
 *   for PT_BVH_WIDE_DEVICE (the tree built on the device, milliseconds), or on the device at
 *   first use once the scene's objects have been updated (pt_scene_update_objects: a dynamic
 *   scene; PT_WIDE_BUILD=host / device in the environment overrides).
 * leaf_batch / shade_batch: wavefront thresholds in lanes (0 = default).
 * flags: PT_RENDER_IDENTITY_ORDER disables the longest-tile-first launch order;
 *   PT_RENDER_ACCUMULATE adds the frame to the film's running sums (progressive rendering,
 *   the headless counterpart of the reference's interactive loop renderToGL/renderBySurface,
 *   main.cu:307-340, 489-528) and outputs sqrt(all accumulated samples' sum / their count);
 *   compat mode continues the film's XORWOW streams, sample mode continues the sample index.
 *   pt_film_clear() restarts the accumulation (e.g. after pt_camera_move).  At most 2^24 - 1
 *   accumulated samples per pixel.
 * out_format: PT_OUT_RGB32F (3 floats per pixel), PT_OUT_RGBA8 (4 bytes per pixel, quantised on
 *   the device exactly like PngImage::saveColor, png_image.h:24-30: (uint8)(clamp(c,0,0.999)*256),
 *   alpha 255; rows in film order, row 0 = bottom, pt_write_png_rgba8 flips them) or
 *   PT_OUT_RGBA8_SURFACE (renderBySurface's conversion, main.cu:327-331: (unsigned)(c*255) in an
 *   8-bit field).  For the 8-bit formats `out_rgb` points to n_pixels x 4 bytes. */
enum { PT_KERNEL_DEFAULT = 0, PT_KERNEL_SIMPLE = 1, PT_KERNEL_WAVEFRONT = 2, PT_KERNEL_WIDE = 3 };
enum { PT_RNG_COMPAT = 0, PT_RNG_SAMPLE = 1 };
enum { PT_OUT_RGB32F = 0, PT_OUT_RGBA8 = 1, PT_OUT_RGBA8_SURFACE = 2 };
#define PT_RENDER_IDENTITY_ORDER 1
#define PT_RENDER_ACCUMULATE 2
typedef struct {
    int32_t kernel, leaf_batch, shade_batch, flags;
    int32_t rng, chunk, out_format, reserved1;
} pt_render_opts;
int pt_render_ex(pt_scene* scene, pt_film* film, const pt_camera* cam, int spp, int max_depth,
                 float* out_rgb, int out_on_device, void* stream, const pt_render_opts* opts,
                 pt_stats* stats);
/* Work counters and kernel time of the film's last pt_render / pt_render_ex; waits for that
 * frame to finish.  Reports PT_ERR_STATE if a traversal guard tripped in it (corrupt tree). */
int pt_film_stats(pt_film* film, pt_stats* stats);
/* Re-initialise the film's streams to their initRandom state (asynchronous on `stream`). */
int pt_film_reset(pt_film* film, void* stream);
/* Progressive rendering: zero the film's accumulated sums (asynchronous on `stream`); the number
 * of samples per pixel accumulated so far. */
int pt_film_clear(pt_film* film, void* stream);
int pt_film_accumulated(pt_film* film, int64_t* samples);
void pt_film_destroy(pt_film* film);
void pt_scene_destroy(pt_scene* scene);   /* replaces clearWorldStates (main.cu:451-460) */

#ifdef __cplusplus
}
#endif
#endif
