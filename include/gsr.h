/*
 * gsr.h -- C ABI of the MI355X-native Gaussian-splat forward rasterizer.
 *
 * This library is the drop-in for ONE path of Lucasmogsan/GSViewer: the
 * per-frame forward rasterization of a static Gaussian set for one camera,
 * i.e. what `render/renderer_cuda.py:230-243` hands to the third-party
 * `diff_gaussian_rasterization.GaussianRasterizer`, with the arithmetic of the
 * reference's OpenGL path (`shaders/gau_vert.glsl`, `shaders/gau_frag.glsl`,
 * GL blend state `render/renderer_ogl.py:178-180`).
 *
 * Conventions
 *  - every pointer argument named *_dev is DEVICE memory (HIP, the caller's
 *    device); everything else is host memory.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *  - functions return GSR_OK (0) or a negative gsr_status; the message of the
 *    most recent failure on the calling thread is gsr_last_error().
 *  - matrices are float[16] ROW-MAJOR math matrices (M[r*4+c]), i.e. exactly
 *    the NumPy arrays the reference builds (`util.py:61-93`) before
 *    `util.set_uniform_mat4` transposes them for the column-major GL upload
 *    (`util.py:364-375`).
 *
 * Thread safety: a gsr_scene is immutable after creation and may be rendered
 * concurrently from several gsr_context objects (one per stream). A
 * gsr_context must not be used by two threads at once.
 */
#ifndef GSR_H_
#define GSR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 7

typedef enum gsr_status {
    GSR_OK = 0,
    GSR_ERR_INVALID = -1,   /* bad argument (null pointer, size, layout) */
    GSR_ERR_HIP = -2,       /* HIP runtime error (launch / alloc / copy)  */
    GSR_ERR_NOMEM = -3,     /* device allocation failed                   */
    GSR_ERR_OVERFLOW = -4   /* a capacity would exceed 2^31 entries, or a frame's
                               tile instances 2^32 - 1 (the frame fails; the context
                               renders its next one)                     */
} gsr_status;

typedef struct gsr_scene gsr_scene;      /* static Gaussian set, SoA in HBM   */
typedef struct gsr_context gsr_context;  /* per-stream frame workspace        */

/* Camera for one frame.
 * Replaces the uniforms view_matrix / projection_matrix / cam_pos /
 * hfovxy_focal (gau_vert.glsl:47-50, uploaded by renderer_ogl.py:282-292)
 * and the viewmatrix/projmatrix/campos/tanfov fields of the raster settings
 * (renderer_cuda.py:196-213). */
typedef struct gsr_camera {
    float view[16];          /* V: world -> GL camera (lookAt, util.py:61-76)      */
    float proj[16];          /* P: GL perspective, z_ndc in [-1,1] (util.py:78-93) */
    float campos[3];         /* camera position in world space                      */
    float hfovxy_focal[3];   /* tan(fovx/2), tan(fovy/2), focal (util.py:181-185)   */
    int32_t width, height;   /* image size in pixels                                */
} gsr_camera;

/* Appearance / culling state: the remaining uniforms of gau_vert.glsl:51-67
 * and the OGL renderer setters (renderer_ogl.py:246-318). */
typedef struct gsr_settings {
    float scale_modifier;        /* gaussian_scale_factor (set_scale_modifier)           */
    float screen_scale;          /* screen_display_scale_factor (set_screen_scale_factor) */
    int32_t render_mod;          /* render_mod: 0..3 SH degree cap (>=3: full), -1 billboard
                                    normal, -2 normal, -3 depth, -4 billboard, -5 flat ball,
                                    -6 gaussian ball (gs_elements_control.py:175 maps UI) */
    float dc_factor;             /* adjust_dc_features                                    */
    float extra_factor;          /* adjust_extra_features                                 */
    float color_scale[3];        /* color_scale_factors (update_color_factor)             */
    float rot_modifier[4];       /* quaternion uniform (x,y,z,w) (set_rot_modifier)       */
    float light_rotation[3];     /* degrees about X,Y,Z (set_light_rotation)              */
    int32_t enable_aabb;         /* set_enable_aabb                                       */
    int32_t enable_obb;          /* set_enable_obb                                        */
    float cube_rotation[9];      /* row-major R (set_cube_rotation, util.py:453-479)      */
    float cube_min[3];           /* cubeMin                                               */
    float cube_max[3];           /* cubeMax                                               */
    float points_center[3];      /* points_center (set_points_center)                     */
    float bg[3];                 /* background (clear colour (0,0,0), main.py:197)        */
    float t_min;                 /* stop a pixel once transmittance < t_min (0 = never)   */
    int32_t out_layout;          /* 0: planar [3,H,W] (rasterizer output, renderer_cuda.py:234)
                                    1: interleaved [H,W,3] (renderer_cuda.py:245)          */
    int32_t blend;               /* GSR_BLEND_FLOAT: front-to-back in float (t_min applies);
                                    GSR_BLEND_UNORM8: the viewer's RGBA8 framebuffer -- GL
                                    SRC_ALPHA/ONE_MINUS_SRC_ALPHA blending in draw order,
                                    every blend result rounded to 8 bits (renderer_ogl.py:178-180,
                                    main.py:197-198); output values are k/255 (t_min unused) */
} gsr_settings;

#define GSR_BLEND_FLOAT 0
#define GSR_BLEND_UNORM8 1

/* Per-frame statistics of the last gsr_render on a context. */
typedef struct gsr_frame_stats {
    int64_t n_gaussians;     /* N                                          */
    int64_t n_visible;       /* passed box + frustum cull                  */
    int64_t n_instances;     /* (splat, 16x16 tile) pairs composited       */
    int32_t tiles_x, tiles_y;
} gsr_frame_stats;

int gsr_abi_version(void);
const char* gsr_last_error(void);
/* 16 hex digits of the digest of the sources the library was built from
 * (gsviewer_amd/_srcid.py); the Python binding refuses a library older than
 * the tree it sits in. */
const char* gsr_source_digest(void);

/* Reference start-up uniform state (main.py:128-137, renderer_ogl.py:183-187). */
void gsr_settings_default(gsr_settings* s);

/* Create a scene from device arrays in the GaussianData layout
 * (util_gau.py:10-42, GaussianDataCUDA renderer_cuda.py:60-101):
 *   xyz [n,3], rot [n,4] (w,x,y,z), scale [n,3] (activated), opacity [n,1]
 *   (activated), sh [n, sh_dim] coefficient-major RGB-interleaved.
 * sh_dim is GaussianData.sh_dim (3, 12, 27 or 48). The data is repacked once
 * into library-owned SoA planes; inputs may be freed afterwards. Ordered on
 * `stream`. Replaces OpenGLRenderer.update_gaussian_data (renderer_ogl.py:235)
 * and CUDARenderer.update_gaussian_data (renderer_cuda.py:147). */
int gsr_scene_create(const float* xyz_dev, const float* rot_dev, const float* scale_dev,
                     const float* opacity_dev, const float* sh_dev, int64_t n, int32_t sh_dim,
                     void* stream, gsr_scene** out);

/* Same, from the flat() AoS record buffer the OGL path uploads as SSBO 0:
 * [n, 11 + sh_dim] floats (util_gau.py:40-42, gau_vert.glsl:28-42). */
int gsr_scene_create_flat(const float* flat_dev, int64_t n, int32_t sh_dim, void* stream,
                          gsr_scene** out);

int gsr_scene_destroy(gsr_scene* scene);
int64_t gsr_scene_count(const gsr_scene* scene);
int32_t gsr_scene_sh_dim(const gsr_scene* scene);

/* Frame workspace. Device buffers grow on demand and are reused; growth
 * never frees (hipFree would synchronise the device): the old blocks are
 * released with the context. */
int gsr_context_create(gsr_context** out);
int gsr_context_destroy(gsr_context* ctx);
/* Size every workspace buffer up front for scenes of up to n Gaussians, frames
 * of up to width x height and up to max_instances (splat, tile) instances per
 * frame (<= 0: 4 n), so that frames within those bounds allocate nothing.
 * The reference sizes its GL buffers once per scene in update_gaussian_data
 * (renderer_ogl.py:235-242) and CUDARenderer keeps its tensors resident
 * (renderer_cuda.py:147-150).
 * Host-side sizing only: nothing is enqueued on `stream` (kept for the ABI),
 * so frames may begin on any stream right after it returns with no
 * synchronisation.  The context's first frame zeroes its completion counter
 * on that frame's own stream. */
int gsr_context_reserve(gsr_context* ctx, int64_t n, int32_t width, int32_t height, int64_t max_instances,
                        void* stream);
/* Device bytes the context holds now (retired blocks excluded), or < 0 on
 * error; *n_allocations (nullable) = device allocations made so far. */
int64_t gsr_context_workspace(gsr_context* ctx, int64_t* n_allocations);

/* Caller-provided workspace ("writes into caller-provided output
 * and workspace"; the reference's caller owns every buffer it hands the
 * rasterizer, renderer_cuda.py:94-100, 230-243).
 * gsr_workspace_size: device bytes one context needs for scenes of <= n
 * Gaussians, frames of <= width x height and <= max_instances tile instances
 * (<= 0: 4 n), or < 0 (a GSR_ERR_*) on bad arguments.  No HIP call: it runs
 * without a GPU.
 * gsr_context_attach_workspace: a new context takes ws_dev[0, ws_bytes) (device
 * memory the caller owns and keeps alive until gsr_context_destroy) for all of
 * its buffers instead of allocating, sized for the same bounds; GSR_ERR_NOMEM
 * if ws_bytes < gsr_workspace_size(...).  Frames within the bounds then never
 * allocate device memory; a frame beyond them fails with GSR_ERR_NOMEM instead
 * of growing (spare bytes past gsr_workspace_size are never carved later, so
 * gsr_context_workspace stays constant).  Only a context that holds no buffers
 * yet can attach one.  Like gsr_context_reserve it enqueues nothing on
 * `stream`: the first frame may begin on any stream without a sync. */
int64_t gsr_workspace_size(int64_t n, int32_t width, int32_t height, int64_t max_instances);
int gsr_context_attach_workspace(gsr_context* ctx, void* ws_dev, size_t ws_bytes, int64_t n, int32_t width,
                                 int32_t height, int64_t max_instances, void* stream);

/* Render one frame: cull + project + SH (preprocess), depth radix sort,
 * tile binning + stable tile sort, 16x16-tile front-to-back compositing.
 * out_image_dev: float32, 3*H*W, layout per settings->out_layout, row 0 = top.
 * radii_dev: optional int32 [n]; 0 for culled Gaussians, else
 *            ceil(max(quad half-width, half-height)) in pixels.
 * Replaces CUDARenderer.draw's rasterizer call (renderer_cuda.py:230-243) and
 * OpenGLRenderer.draw + sort_and_update (renderer_ogl.py:263-268, 406-412).
 * Its depth sort runs 3 radix passes (GSR_DEPTH_PASSES_ALONE, 3 or 4, read at
 * context creation); frames begun with gsr_render_begin* run 4 narrower ones,
 * whose kernels fit beside other views' compositing.  Same order either way. */
int gsr_render(gsr_context* ctx, const gsr_scene* scene, const gsr_camera* cam,
               const gsr_settings* settings, float* out_image_dev, int32_t* radii_dev,
               void* stream);

/* gsr_render in two halves, for callers that keep several independent views
 * in flight (one context and stream each).  _begin enqueues culling,
 * preprocess and the depth sort and returns at once; _finish waits (on the
 * host) for the frame's visible/instance counts and enqueues the rest.  A
 * caller begins the next view's frame before finishing this one, so the
 * host never idles while the GPU could take more work.  One frame per
 * context may be pending; _finish takes the same stream.  A context's buffers
 * belong to the stream of its last frame until that frame completes: before
 * using the context on another stream, synchronise (or make the new stream
 * wait for the old one). */
int gsr_render_begin(gsr_context* ctx, const gsr_scene* scene, const gsr_camera* cam,
                     const gsr_settings* settings, float* out_image_dev, int32_t* radii_dev,
                     void* stream);
int gsr_render_finish(gsr_context* ctx, void* stream);

/* Several views of ONE scene begun together (stereo, multi-camera capture, a
 * batch of views in flight): the cull and preprocess of all k views
 * (k <= GSR_MAX_VIEWS, one context each, same settings) read the scene once,
 * in one pass enqueued on `stream`.  Then, per view, after its own stream has
 * been made to wait for `stream` (an event), gsr_render_begin_sort(ctx, its
 * stream) enqueues the depth sort, and gsr_render_finish(ctx, its stream)
 * completes the frame as for gsr_render_begin.  Results are identical to
 * rendering each view alone.  cams[k], outs[k], radii[k] (radii may be NULL,
 * or hold NULL entries). */
#define GSR_MAX_VIEWS 8
int gsr_render_begin_views(gsr_context* const* ctxs, int32_t k, const gsr_scene* scene,
                           const gsr_camera* cams, const gsr_settings* settings,
                           float* const* out_images_dev, int32_t* const* radii_dev, void* stream);
int gsr_render_begin_sort(gsr_context* ctx, void* stream);
/* The depth sorts of k views begun by one gsr_render_begin_views, in one
 * launch per radix step on `stream` (which then also takes their
 * gsr_render_finish). */
int gsr_render_begin_sorts(gsr_context* const* ctxs, int32_t k, void* stream);
/* gsr_render_finish for k begun frames pending on the same `stream` (e.g. the
 * views of one gsr_render_begin_sorts): binning, tile sort, compositing and
 * merge run as one launch per step for all k.  The views must share frame
 * size, t_min, background, output layout, fragment mode and chunk length.  A group's frames are
 * composited in chunks of GSR_CHUNK_VIEWS instances (default 3072: views in flight fill the chip
 * while a deep tile's chunk runs), a frame finished alone in chunks of GSR_CHUNK (default 192:
 * latency); both read when the context is created.  Chunks are dispatched longest first (full
 * chunks, then GSR_LEN_CLASSES - 1 length classes of the last chunks, default 8), a group's
 * views interleaved class by class (GSR_VIEWS_INTERLEAVE=0: view after view); a group dispatches
 * every tile's first chunk before any later chunk (GSR_FIRST_MAJOR=0: full chunks first), so a
 * deep tile saturated by its first chunk skips the rest.
 * Results are identical to k gsr_render_finish calls (and independent of the dispatch order).
 * Once the arguments are validated every view's frame is consumed: an error
 * after that point (a wait timeout, GSR_ERR_NOMEM beyond a caller workspace's
 * bounds) ends all k frames, and each context can begin its next one. */
int gsr_render_finish_views(gsr_context* const* ctxs, int32_t k, void* stream);

/* Host wait, without finishing, until the begun frame of `ctx` has published its
 * counts (its cull + preprocess has completed on the GPU).  The frame stays
 * pending; finish it as usual.  (Staggering a pipeline's groups with it --
 * each group's preprocess waited for before the next group begins -- measured
 * slower: profiles/r4_s30.)  Same deadline and failure rules as the finish's
 * own wait; GSR_ERR_INVALID when no frame is pending. */
int gsr_render_wait_counts(gsr_context* ctx);

int gsr_context_stats(const gsr_context* ctx, gsr_frame_stats* out);

/* Back-to-front Gaussian order for a view matrix: the renderer_ogl
 * _sort_gaussian_{cpu,torch,cupy} service (renderer_ogl.py:16-59) as a device
 * radix sort. Writes index_dev[n] (int32, ascending view-space z; ties keep
 * ascending index). */
int gsr_sort_depth(gsr_context* ctx, const gsr_scene* scene, const float view[16],
                   int32_t* index_dev, void* stream);

/* Test hook: stable sort of n uint32 keys < 2^bits (values = 0..n-1) with
 * the frame's radix sort, in `passes` passes of ceil(bits/passes) <= 11 bits.
 * Asynchronous on `stream`, like gsr_render. */
int gsr_debug_sort_pairs(gsr_context* ctx, const uint32_t* keys_dev, int64_t n, int32_t bits, int32_t passes,
                         uint32_t* keys_out_dev, uint32_t* vals_out_dev, void* stream);

/* Optional per-stage GPU timing with HIP events recorded on the render stream
 * (no extra synchronisation in the frame; accumulated lazily).
 * Stages: cull (+ visible-count scan), preprocess, depth sort, binning
 * (tile counts, scan, instance write), tile sort, tile ranges, composite, and
 * `sync` = GPU idle time while the host reads the visible/instance counts. */
enum { GSR_STAGE_CULL = 0, GSR_STAGE_PREPROCESS = 1, GSR_STAGE_DEPTH_SORT = 2, GSR_STAGE_BINNING = 3,
       GSR_STAGE_TILE_SORT = 4, GSR_STAGE_RANGES = 5, GSR_STAGE_COMPOSITE = 6, GSR_STAGE_SYNC = 7,
       GSR_STAGE_MERGE = 8, GSR_NUM_STAGES = 9 };
/* enable: 0 off, 1 per-stage events of this context's single-view frames,
 * 2 events around the compositing launch of every group this context leads
 * (ctxs[0] of gsr_render_finish_views; gsr_context_group_times).  Resets the
 * accumulators. */
int gsr_context_set_profiling(gsr_context* ctx, int32_t enable);
/* Sum of per-stage milliseconds over the profiled frames since the last reset
 * (waits for the last profiled frame's events). */
int gsr_context_stage_times(gsr_context* ctx, double* ms_out /* [GSR_NUM_STAGES] */, int64_t* frames_out);
/* Profiling mode 2: summed milliseconds of the group compositing launches
 * (k_composite_views) measured by HIP events on the group's stream, the
 * number of launches and the views they composited, and (span_ms, nullable)
 * the summed in-kernel spans of the same launches: first block start to last
 * wave end by the 100 MHz constant clock (s_memrealtime), i.e. the kernel's
 * execution without the time its dispatch waited behind other streams'
 * work.  Synchronises the device. */
int gsr_context_group_times(gsr_context* ctx, double* composite_ms, int64_t* launches, int64_t* views,
                            double* span_ms);
/* Profiling mode 2: the in-kernel span of each recorded compositing launch,
 * (first block start, last wave end) in ticks of the 100 MHz constant clock
 * (device-wide, so spans of different contexts' launches compare), written
 * as pairs to spans_out[2 * i], [2 * i + 1] for i < max_spans.  Returns the
 * number of recorded launches (>= 0; may exceed max_spans) or a negative
 * gsr_status.  Synchronises the device. */
int64_t gsr_context_group_spans(gsr_context* ctx, uint64_t* spans_out, int64_t max_spans);

/* Host time spent inside gsr_render on this context since creation, in ms:
 * [0] enqueue before the wait for the frame's counts, [1] that wait,
 * [2] enqueue after it; *frames_out = number of frames. */
int gsr_debug_host_times(const gsr_context* ctx, double ms_out[3], int64_t* frames_out);

/* Test hook: keep `stream` busy for `microseconds` (<= 5 s) with one wave
 * that sleeps until the time has passed (exercises the bounded host wait:
 * GSR_WAIT_TIMEOUT_MS, default 2000, after which gsr_render_finish returns
 * GSR_ERR_HIP and the context is marked failed). */
int gsr_debug_stall(void* stream, uint32_t microseconds);

/* Test hook: copy an internal array of the last gsr_render on `ctx` into
 * dst_dev (device memory, at most max_bytes). Returns the number of bytes
 * copied (>= 0) or a negative gsr_status.  what:
 *   GSR_DEBUG_RECORDS      48-B splat records by slot.  Culling fused into the
 *                          preprocess (the default; GSR_FUSED_CULL=0 at context
 *                          creation selects the separate cull): one slot per
 *                          Gaussian, slot n-1-id, N records (culled slots hold
 *                          no record).  Separate cull: compacted, slot s = the
 *                          s-th visible Gaussian in DESCENDING id order, V records.
 *   GSR_DEBUG_DEPTH_ORDER  uint32 record slots, front-to-back.  A frame alone
 *                          (gsr_render) sorts only the top 16 bits of its depth
 *                          key range (GSR_DEPTH_COARSE, 0 = exact): equal coarse
 *                          keys in slot order; the tile lists are exact.  A
 *                          group's frames sort exactly.
 *   GSR_DEBUG_TILE_RANGES  uint32 pairs [begin, end) per 16x16 tile (row-major tiles)
 *   GSR_DEBUG_TILE_LIST    uint32 record slots of all (tile, splat) instances, by tile then depth */
enum { GSR_DEBUG_RECORDS = 0, GSR_DEBUG_DEPTH_ORDER = 1, GSR_DEBUG_TILE_RANGES = 2, GSR_DEBUG_TILE_LIST = 3 };
int64_t gsr_debug_copy(const gsr_context* ctx, int32_t what, void* dst_dev, int64_t max_bytes, void* stream);

/* Test / A-B hook: the value of a stage-form knob of `ctx` as read from the
 * environment at gsr_context_create, or the form the context's last frame
 * took.  Knobs: "rect_payload" (0 = GSR_NO_RECT_PAYLOAD), "fused_cull",
 * "bin_fused", "depth_coarse_alone", "chunk", "chunk_target", "chunk_views",
 * "tail_merge_alone", "tail_merge_group", "first_major", "first_major_alone",
 * "bound_alone" (GSR_BOUND_ALONE: every frame alone with t_min > 0 takes the deep
 * form's first-major order and cross-chunk bound; measured slower at C2),
 * "chunk_single" (GSR_CHUNK_SINGLE=0: a frame alone's chunk descriptors by the
 * count + write launches instead of one block).
 * Last frame: "frame_packed" (its depth sort carried the packed tile rects),
 * "frame_coarse" (its depth sort's coarse bits, 0 = exact), "frame_chunk" (its
 * compositing chunk length; 0 for the RGBA8 framebuffer), "frame_deep" (1: the
 * deep-frame form: longer chunks and the cross-chunk transmittance bound).
 * GSR_ERR_INVALID for an unknown name.  No GPU work. */
int gsr_context_knob(const gsr_context* ctx, const char* name, int64_t* value);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H_ */
