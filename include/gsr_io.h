/* gsr_io.h -- scene ingestion and export around the rasterization hot path
 * (SURVEY.md §8(f) rows 2 and 3).  Same conventions as gsr.h: plain C ABI,
 * 0 / negative gsr_status returns, message in gsr_last_error().
 *
 * Row 2, native PLY ingestion, replaces the parse half of util_gau.load_ply
 * (util_gau.py:236-305: PlyData.read + the pandas column gathers).  The
 * activations (exp of scales, sigmoid of opacity, quaternion normalisation,
 * :297-303) stay with the caller.  gsviewer_amd/ply.py applies them with the
 * reference's own NumPy expressions, so the loaded scene is bit-identical.
 *
 * Row 3, GPU box mask and compaction for export, replaces the filtering half
 * of util_gau.export_ply (util_gau.py:388-430) plus gsconverter's
 * crop_by_bbox (tools/gsconverter/utils/base_converter.py:175-191) and its
 * 3dgs writer (format_3dgs.py:66-87, main.py:108-110).
 */
#ifndef GSR_IO_H
#define GSR_IO_H

#include <stdint.h>

#include "gsr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* PLY body encodings. */
enum { GSR_PLY_BINARY_LE = 0, GSR_PLY_BINARY_BE = 1, GSR_PLY_ASCII = 2 };

typedef struct gsr_ply_info {
    int64_t n;            /* rows of the "vertex" element */
    int32_t sh_dim;       /* 3 (no f_rest_*: degree 0) or 48 (45 f_rest_*: degree 3) */
    int32_t format;       /* GSR_PLY_* */
    int32_t n_properties; /* properties of the vertex element */
    int32_t row_bytes;    /* bytes per binary row (0 for ascii) */
    int64_t body_offset;  /* byte offset of the first row */
} gsr_ply_info;

/* Parse the header.  Errors, matching where load_ply itself would fail:
 * no vertex element, a missing x/y/z/opacity/f_dc_0..2 property, f_rest_*
 * counts other than 0 or 45 (load_ply's reshape to (N, 3, 15),
 * util_gau.py:287-289), or a list property in the vertex element. */
int gsr_ply_probe(const char* path, gsr_ply_info* info);

/* Read the raw (pre-activation) vertex columns into host float32 arrays:
 * xyz [n,3], rot [n,4] (rot_* sorted by suffix), scale [n,3] (scale_* sorted),
 * opacity [n,1], sh [n,sh_dim].  sh is in load_ply's layout: f_dc_0..2, then
 * f_rest reshaped (3, K-1) and transposed, i.e. sh[3 + 3j + c] = f_rest[c*(K-1) + j].
 * Other property types are converted to float32.  n_threads <= 0 means "all
 * hardware threads". */
int gsr_ply_read(const char* path, float* xyz, float* rot, float* scale, float* opacity, float* sh,
                 int32_t n_threads);

/* The viewer's "Open ply" step straight into a device scene: util_gau.load_ply
 * (util_gau.py:236-305), then GaussianData.scale_data(scale_to_interval)
 * (util_gau.py:44-53; the viewer uses 5.0, gs_elements_control.py:41-42; <= 0
 * skips it) and points_center (np.mean(xyz, axis=0), :44), then the SoA
 * repack of update_gaussian_data.  The vertex rows are parsed by host threads
 * in chunks into pinned buffers and copied while the next chunk is parsed;
 * the activations, the rescale and the mean run on the GPU in the
 * reference's float32 order (xyz, rot, sh bit-identical to load_ply +
 * scale_data; scale and opacity within a few ulps: NumPy's float32 exp is its
 * own SIMD polynomial).  Synchronous on `stream`. */
typedef struct gsr_ply_scene_info {
    int64_t n;
    int32_t sh_dim;
    int32_t pad;
    float points_center[3];  /* after the rescale: set_points_center's value */
    float scale_factor;      /* scale_data's factor (1 when skipped) */
    float bbox_center[3];    /* scale_data's centre (0 when skipped) */
} gsr_ply_scene_info;
int gsr_scene_load_ply(const char* path, float scale_to_interval, int32_t n_threads, void* stream, gsr_scene** out,
                       gsr_ply_scene_info* info);

/* A scene back as flat rows [n, 11 + sh_dim] (util_gau.py:40-42) in device memory. */
int gsr_scene_read_flat(const gsr_scene* scene, float* flat_dev, void* stream);

/* Write rows of `in_path` to `out_path` in gsconverter's 3dgs layout:
 * binary_little_endian; float properties x y z nx ny nz f_dc_0..2
 * f_rest_0..44 opacity scale_0..2 rot_0..3.  Values are copied by name and a
 * property the input lacks is written as 0 (Utility.copy_data_with_prefix_check).
 * rows: ascending host row indices, or NULL for all rows. */
int gsr_ply_write_3dgs(const char* in_path, const char* out_path, const int64_t* rows, int64_t n_rows,
                       int32_t n_threads);

/* Box filter of export_ply (util_gau.py:389-408). */
enum { GSR_BOX_NONE = 0, GSR_BOX_AABB = 1, GSR_BOX_OBB = 2 };
typedef struct gsr_box {
    int32_t mode;        /* GSR_BOX_*; OBB wins when both are enabled, as in export_ply */
    int32_t pad;
    double cube_min[3];  /* AABB: the thresholds points_center + cubeMin (:402, the double offset);
                            OBB: cubeMin.  Either as NumPy computes them from the caller's dtypes. */
    double cube_max[3];  /* likewise for cubeMax */
    double rot_inv[9];   /* OBB: np.linalg.inv(rotation_matrix), row-major */
} gsr_box;

/* points_center = np.mean(xyz, axis=0) of a float32 [n,3] device array,
 * bit-exact: NumPy sums an axis-0 reduction row after row in float32 and
 * divides in float32, so one GPU wave does the same.  Host result, synchronous. */
int gsr_points_center(const float* xyz_dev, int64_t n, float center[3], void* stream);

/* On the GPU, for n points:
 *   mask   = box predicate on (xyz_cur - center) (float32 subtract, float64 compare, :397-405)
 *   bbox   = [min, max] of xyz_orig over the mask (:411-413)
 *   rows   = ascending indices i with xyz_orig[i] inside bbox, inclusive:
 *            the rows gsconverter's crop keeps (base_converter.py:177-184).
 * xyz_cur / xyz_orig: device float32 [n,3] (the current scene, the as-loaded
 * positions).  rows_dev: device int64 [n].  Synchronous.  On return *n_rows
 * holds the count.  *has_bbox is 0 when the mask is empty: export_ply then
 * passes bbox=None, gsconverter crops nothing, and all n rows are kept. */
int gsr_export_select(const float* xyz_cur_dev, const float* xyz_orig_dev, int64_t n, const float center[3],
                      const gsr_box* box, int64_t* rows_dev, int64_t* n_rows, float bbox[6], int32_t* has_bbox,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_IO_H */
