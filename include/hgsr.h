/*
 * hgsr.h — C ABI of the MI355X (gfx950) differentiable Gaussian rasterizer.
 *
 * This is the drop-in boundary for the hot path that Horizon-GS reaches through
 * gsplat (reference gaussian_renderer/render.py:13-14, :40-76, :149-186).  Each
 * entry replaces one gsplat CUDA-extension op; the gsplat-compatible Python
 * surface (horizongs_amd/gsplat_api.py, re-exported by the `gsplat` alias
 * package) binds them with ctypes.
 *
 * Conventions (all entries):
 *   - every pointer is a DEVICE pointer to row-major contiguous memory, allocated
 *     by the caller (the library never allocates); fp32 data, int32 ids/radii,
 *     int64 intersection keys;
 *   - gradient outputs are OVERWRITTEN unless the entry's comment says otherwise
 *     (the raster / projection / SH-coefficient backwards write every element; v_dirs of
 *     hgsr_sh_bwd and the decode backward's input / weight gradients accumulate (+=) into
 *     caller-zeroed buffers, as noted at each entry);
 *   - work is enqueued on `stream` (a hipStream_t; NULL = default stream) and the
 *     call returns without synchronising;
 *   - return 0 (HGSR_OK) or a negative status; hgsr_last_error() then holds a
 *     thread-local message.  Data values are not validated (NaN propagates).
 *   - C = cameras, N = Gaussians; per-camera arrays are [C, N, ...]; "flatten ids"
 *     index the [C*N] flattened arrays (gsplat non-packed mode).
 */
#ifndef HGSR_H
#define HGSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* hgsr_stream_t; /* hipStream_t */

enum {
    HGSR_OK = 0,
    HGSR_EINVAL = -1,     /* bad dimensions / unsupported option / null pointer */
    HGSR_ELAUNCH = -2,    /* kernel launch failed */
    HGSR_EWORKSPACE = -3  /* workspace too small */
};

int hgsr_version(void);
const char* hgsr_last_error(void);

/* ---- K1/K2: 3DGS EWA projection ----------------------------------------
 * replaces gsplat.cuda._wrapper.fully_fused_projection (packed=False), called at
 * reference gaussian_renderer/render.py:149-165 and inside gsplat.rasterization
 * (render.py:40-54).  Outputs [C,N] radii (0 = culled), means2d [C,N,2],
 * depths [C,N], conics [C,N,3].  Optionally (tile_counts != NULL) nothing else. */
int hgsr_project3d_fwd(int C, int N, const float* means, const float* quats,
                       const float* scales, const float* viewmats, const float* Ks,
                       int width, int height, float eps2d, float near_plane,
                       float far_plane, float radius_clip, int32_t* radii, float* means2d,
                       float* depths, float* conics, hgsr_stream_t stream);

/* vjp of the above: writes (overwrites) v_means [N,3], v_quats [N,4], v_scales [N,3];
 * v_scales_in (nullable [N,3]): another consumer's gradient of the same scales (the loss
 * head's scale regulariser), added into v_scales in the same pass; v_means_in (nullable
 * [N,3]): likewise for the means (the SH colour step's view directions, hgsr_sh_rgb_bwd). */
int hgsr_project3d_bwd(int C, int N, const float* means, const float* quats,
                       const float* scales, const float* viewmats, const float* Ks,
                       int width, int height, float eps2d, const int32_t* radii,
                       const float* conics, const float* v_means2d, const float* v_depths,
                       const float* v_conics, float* v_means, float* v_quats, float* v_scales,
                       const float* v_scales_in, const float* v_means_in, hgsr_stream_t stream);

/* ---- K1'/K10: 2DGS surfel projection -------------------------------------
 * replaces fully_fused_projection_2dgs (render.py:171-186 and inside
 * gsplat.rasterization_2dgs).  Outputs radii, means2d, depths,
 * ray_transforms [C,N,3,3] (row-major K*[R*Rq*diag(sx,sy,1) | t]) and
 * camera-facing normals [C,N,3]. */
int hgsr_project2d_fwd(int C, int N, const float* means, const float* quats,
                       const float* scales, const float* viewmats, const float* Ks,
                       int width, int height, float near_plane, float far_plane,
                       float radius_clip, int32_t* radii, float* means2d, float* depths,
                       float* ray_transforms, float* normals, hgsr_stream_t stream);

/* vjp of the above: writes (overwrites) v_means, v_quats, v_scales (v_scales[:,2] = 0);
 * v_scales_in (nullable): added into v_scales, as in hgsr_project3d_bwd. */
int hgsr_project2d_bwd(int C, int N, const float* means, const float* quats,
                       const float* scales, const float* viewmats, const float* Ks,
                       int width, int height, const int32_t* radii,
                       const float* ray_transforms, const float* v_means2d,
                       const float* v_depths, const float* v_ray_transforms,
                       const float* v_normals, float* v_means, float* v_quats,
                       float* v_scales, const float* v_scales_in, hgsr_stream_t stream);

/* ---- K3: spherical-harmonics colour --------------------------------------
 * replaces gsplat spherical_harmonics (used by rasterization when sh_degree is
 * not None; SH2 configs).  dirs [n,3] (unnormalised), coeffs [n,K,3],
 * masks [n] (uint8, nullable) -> colors [n,3] (written).  Basis polynomials of
 * reference utils/sh_utils.py:57-112, degree <= 3. */
int hgsr_sh_fwd(int degree, int K, int64_t n, const float* dirs, const float* coeffs,
                const uint8_t* masks, float* colors, hgsr_stream_t stream);
/* writes v_coeffs [n,K,3]; accumulates v_dirs [n,3] (nullable). */
int hgsr_sh_bwd(int degree, int K, int64_t n, const float* dirs, const float* coeffs,
                const uint8_t* masks, const float* v_colors, float* v_coeffs, float* v_dirs,
                hgsr_stream_t stream);
/* rasterization()'s colour path for sh_degree != None in one call each way
 * (gsplat rendering.py as HorizonGS calls it from gaussian_renderer/render.py:40-54:
 * dirs = means - campos[c]; colors = spherical_harmonics(sh_degree, dirs, coeffs,
 * masks = radii > 0); colors = clamp_min(colors + 0.5, 0)).  means [N,3], campos [C,3],
 * coeffs [N,K,3] (shared = 1) or [C,N,K,3], radii [C,N] -> colors [C,N,3] (written).
 * The backward writes v_coeffs (summed over cameras when shared) and v_means [N,3]
 * (nullable; overwritten, = the gradient through dirs).  The backward takes K <= 16
 * (degree <= 3 coefficient rows, staged through LDS); HGSR_EINVAL otherwise.  viewmats
 * (nullable, [C,4,4] world-to-camera, row-major): the camera centres -R^T t are computed in
 * the kernels from them instead of read from campos (which may then be NULL). */
int hgsr_sh_rgb_fwd(int degree, int C, int N, int K, const float* means, const float* campos,
                    const float* viewmats, const float* coeffs, int shared, const int32_t* radii,
                    float* colors, hgsr_stream_t stream);
int hgsr_sh_rgb_bwd(int degree, int C, int N, int K, const float* means, const float* campos,
                    const float* viewmats, const float* coeffs, int shared, const int32_t* radii,
                    const float* v_colors, float* v_coeffs, float* v_means, hgsr_stream_t stream);

/* ---- K5/K6/K7: tile intersection, sort, tile offsets ---------------------
 * Replaces gsplat isect_tiles(sort=True) + cub DeviceRadixSort + isect_offset_encode
 * with a tile-bucketed binning:
 *   stage 1 (hgsr_isect_count): tile rectangle per Gaussian -> tiles_per_gauss
 *     [C,N]; per-block tile histograms; isect_offsets [C, tile_h, tile_w]
 *     (exclusive scan over (camera, tile) bins = gsplat isect_offset_encode);
 *     `info` (device, 2 x int64) = {n_isects, largest bin}.
 *   stage 2 (hgsr_isect_emit_sorted, after the host reads info[0]): scatter
 *     (depth, id) keys into their bins and sort each bin; writes the SORTED
 *     isect_ids [n_isects] (cam<<(32+tile_bits) | tile<<32 | depth bits) and
 *     flatten_ids [n_isects], bit-identical to a stable radix sort of gsplat's
 *     Gaussian-major emission.
 * The same `ws1` must be passed to both stages.
 * Deferred count (isect_info != NULL, the `info` of stage 1 allocated as 3 x int64): stage 2
 *   is enqueued BEFORE the host reads the count, n_isects / max_bin being the caller's
 *   capacities (isect_ids / flatten_ids / ws2 sized for them).  The kernels read the true
 *   count from info[0..1]; when it exceeds a capacity they emit nothing and set info[2] = 1
 *   (else 0), and hgsr_raster{3,2}d_fwd_packed given the same info composite nothing.  The
 *   caller checks the count it copies back and re-runs stage 2 at the exact size on overflow.
 *   Otherwise the first info[0] entries of isect_ids / flatten_ids are the sorted result. */
size_t hgsr_isect_ws1_bytes(int C, int N, int tile_w, int tile_h);
size_t hgsr_isect_ws2_bytes(int64_t n_isects, int64_t max_bin);
int hgsr_isect_count(int C, int N, const float* means2d, const int32_t* radii, int tile_size,
                     int tile_w, int tile_h, int32_t* tiles_per_gauss, int32_t* isect_offsets,
                     int64_t* info, void* ws1, size_t ws1_bytes, hgsr_stream_t stream);
int hgsr_isect_emit_sorted(int C, int N, const float* means2d, const int32_t* radii,
                           const float* depths, int tile_size, int tile_w, int tile_h,
                           const int32_t* isect_offsets, int64_t n_isects, int64_t max_bin,
                           int64_t* isect_ids, int32_t* flatten_ids, void* ws1,
                           size_t ws1_bytes, void* ws2, size_t ws2_bytes, int64_t* isect_info,
                           hgsr_stream_t stream);
/* gsplat isect_tiles(sort=False): Gaussian-major emission; cum_tiles = inclusive
 * prefix sum of tiles_per_gauss over the flattened [C*N]. */
int hgsr_isect_emit_unsorted(int C, int N, const float* means2d, const int32_t* radii,
                             const float* depths, int tile_size, int tile_w, int tile_h,
                             const int64_t* cum_tiles, int64_t* isect_ids,
                             int32_t* flatten_ids, hgsr_stream_t stream);
/* gsplat isect_offset_encode on already-sorted ids -> offsets [C, tile_h, tile_w]. */
int hgsr_isect_offset_encode(int64_t n_isects, const int64_t* isect_ids, int C, int tile_w,
                             int tile_h, int32_t* offsets, hgsr_stream_t stream);

/* ---- K8/K9: 3DGS tile rasterization ---------------------------------------
 * replaces gsplat rasterize_to_pixels (packed=False, tile_size=16, D <= 4 per
 * call; callers chunk wider channel counts).  colors [C*N, D], opacities [C*N],
 * backgrounds [C, D] nullable.  Outputs render_colors [C,H,W,D],
 * render_alphas [C,H,W,1], last_ids [C,H,W].  ws: caller scratch of
 * hgsr_raster3d_fwd_ws_bytes() (packed 64-B per-Gaussian raster records, then room for
 * the gradient slots' prefix a training pack writes: 4 B per (camera, Gaussian) + 1 KB). */
size_t hgsr_raster3d_fwd_ws_bytes(int C, int N, int D);
int hgsr_raster3d_fwd(int C, int N, int D, const float* means2d, const float* conics,
                      const float* colors, const float* opacities, const float* backgrounds,
                      int width, int height, int tile_size, int tile_w, int tile_h,
                      const int32_t* isect_offsets, int64_t n_isects,
                      const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                      int32_t* last_ids, void* ws, size_t ws_bytes, hgsr_stream_t stream);
/* writes (overwrites) v_means2d [C*N,2], v_conics [C*N,3], v_colors [C*N,D],
 * v_opacities [C*N]; v_means2d_abs nullable (gsplat absgrad).  fwd_ws: the
 * workspace hgsr_raster3d_fwd filled for the same inputs (its packed records
 * are reused; the backward writes each record's gradient-slot quad, a field the
 * forward does not read), or NULL to pack again.  ws: caller scratch of
 * hgsr_raster3d_bwd_ws_bytes(C, N, D, n_isects, fwd_ws != NULL).
 * Deterministic: every (tile, Gaussian) pair's per-wave partial sums go to the pair's own
 * gradient slot and each Gaussian's slots are summed in one fixed order (no float atomics),
 * so the same inputs give bit-identical gradients on every launch.  The slots follow each
 * Gaussian's tile rectangle in isect_tiles order; this entry finds the rectangles from the
 * lists (flatten_ids must come from isect_tiles: every Gaussian's tiles a full rectangle). */
size_t hgsr_raster3d_bwd_ws_bytes(int C, int N, int D, int64_t n_isects, int reuse_fwd);
int hgsr_raster3d_bwd(int C, int N, int D, const float* means2d, const float* conics,
                      const float* colors, const float* opacities, const float* backgrounds,
                      int width, int height, int tile_size, int tile_w, int tile_h,
                      const int32_t* isect_offsets, int64_t n_isects,
                      const int32_t* flatten_ids, const float* render_alphas,
                      const int32_t* last_ids, const float* v_render_colors,
                      const float* v_render_alphas, float* v_means2d, float* v_conics,
                      float* v_colors, float* v_opacities, float* v_means2d_abs,
                      const void* fwd_ws, void* ws, size_t ws_bytes, hgsr_stream_t stream);

/* Fused channel assembly for gsplat rasterization() (rendering.py: colour/depth
 * concatenation, opacity repeat and the ED normalisation are done in Python there;
 * reference gaussian_renderer/render.py:40-54 calls it with render_mode "RGB+ED").
 * Channels: colors[..., :Dc] (colors [N,Dc] shared over cameras when colors_shared,
 * else [C,N,Dc]) followed by depths [C,N] when depths != NULL; opacities [N] when
 * opacities_shared else [C,N]; backgrounds [C,Dc] (the depth channel has none);
 * expected_depth divides the depth channel by max(alpha, 1e-10).  Outputs
 * render_colors [C,H,W,Dc+(depths?1:0)], render_alphas, last_ids; ws as
 * hgsr_raster3d_fwd_ws_bytes(C, N, Dc + (depths ? 1 : 0)). */
int hgsr_raster3d_fwd_fused(int C, int N, int Dc, const float* means2d, const float* conics,
                            const float* colors, int colors_shared, const float* depths,
                            int expected_depth, const float* opacities, int opacities_shared,
                            const float* backgrounds, int width, int height, int tile_size,
                            int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                            const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                            int32_t* last_ids, void* ws, size_t ws_bytes, hgsr_stream_t stream);
/* hgsr_raster3d_fwd_fused split in two, so the packing runs while the host reads the
 * intersection count (the one host sync of a view): hgsr_raster3d_pack_fused writes the
 * per-Gaussian raster records of the fused channel layout into ws (size as above; it
 * needs no intersection data), hgsr_raster3d_fwd_packed composites from them (with_depth:
 * the records carry the depth channel after the Dc colours).  The records stay valid for
 * hgsr_raster3d_bwd_fused's fwd_ws.  qmask (nullable, hgsr_raster3d_qmask_bytes) receives
 * the forward's per-quadrant culling bits of every tile list, which hgsr_raster3d_bwd_fused
 * (given the same buffer) reads instead of repeating the culling tests; caller-allocated,
 * OVERWRITTEN where the forward visits a tile (the backward reads only those bits).  The
 * buffer starts with the tiles' heaviest-first dispatch order and each tile's latest
 * contributor + 1, which the forward writes; the backward re-sorts the order by the ranges it
 * walks (placement only: no result depends on it).
 * bwd_ws (nullable, 16-B aligned, >= hgsr_raster3d_bwd_ws_bytes(C, N, D, n_isects, 1)): the
 * workspace the backward will get; the forward clears its gradient-slot flags while it
 * composites (HBM is idle there), so hgsr_raster3d_bwd_fused given it with ws_zeroed = 1 skips
 * its memset.
 * isect_info (nullable): the deferred count of hgsr_isect_emit_sorted (n_isects is then the
 * capacity the intersection arrays and qmask were sized for); the quadrant-mask stride is
 * derived from qmask_bytes, so the backward must get the same buffer and size. */
size_t hgsr_raster3d_qmask_bytes(int C, int tile_w, int tile_h, int64_t n_isects);
/* radii (nullable, [C,N] int32, with the tile grid): a backward will follow; the records then
 * carry each (camera, Gaussian)'s gradient-slot base (its isect_tiles rectangle in the grid) and
 * ws the slots' prefix, which hgsr_raster3d_bwd_fused given fwd_slots = 1 uses as they are.
 * tiles_per_gauss (nullable, [C,N] int32): the same rectangles' areas as hgsr_isect_count wrote
 * them for these radii -- the prefix's row sums read them instead of re-deriving the areas. */
int hgsr_raster3d_pack_fused(int C, int N, int Dc, const float* means2d, const float* conics,
                             const float* colors, int colors_shared, const float* depths,
                             const float* opacities, int opacities_shared, const int32_t* radii,
                             const int32_t* tiles_per_gauss, int tile_size, int tile_w, int tile_h,
                             void* ws, size_t ws_bytes, hgsr_stream_t stream);
int hgsr_raster3d_fwd_packed(int C, int N, int Dc, int with_depth, int expected_depth,
                             const float* backgrounds, int width, int height, int tile_size,
                             int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                             const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                             int32_t* last_ids, const void* records, size_t records_bytes,
                             void* qmask, size_t qmask_bytes, void* bwd_ws, size_t bwd_ws_bytes,
                             const int64_t* isect_info, hgsr_stream_t stream);
/* vjp of hgsr_raster3d_fwd_fused: v_colors in the colours' layout (shared colours
 * summed over cameras in camera order), v_depths [C,N] (when depths), v_opacities
 * in the opacities' layout; render_colors is the forward output (needed for ED);
 * qmask (nullable): the buffer hgsr_raster3d_fwd_packed filled for the same lists.
 * radii (nullable, [C,N] int32): the projection's radii the lists were emitted from
 * (isect_tiles(means2d, radii, ...)); given, the gradient slots come from the tile rectangles
 * directly instead of from a pass over the lists.  fwd_slots: fwd_ws came from
 * hgsr_raster3d_pack_fused given these radii (its records carry the slots; only the big
 * entries' piece list is made here).  ws: hgsr_raster3d_bwd_ws_bytes(C, N,
 * Dc + (depths ? 1 : 0), n_isects, fwd_ws != NULL). */
int hgsr_raster3d_bwd_fused(int C, int N, int Dc, const float* means2d, const float* conics,
                            const float* colors, int colors_shared, const float* depths,
                            int expected_depth, const float* opacities, int opacities_shared,
                            const float* backgrounds, int width, int height, int tile_size,
                            int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                            const int32_t* flatten_ids, const float* render_colors,
                            const float* render_alphas, const int32_t* last_ids,
                            const float* v_render_colors, const float* v_render_alphas,
                            float* v_means2d, float* v_conics, float* v_colors, float* v_depths,
                            float* v_opacities, float* v_means2d_abs, const void* fwd_ws, void* ws,
                            size_t ws_bytes, const void* qmask, size_t qmask_bytes, int ws_zeroed,
                            const int32_t* radii, int fwd_slots, hgsr_stream_t stream);

/* ---- K11/K12: 2DGS surfel rasterization -----------------------------------
 * replaces gsplat rasterize_to_pixels_2dgs.  The LAST colour channel is the
 * depth (render_mode RGB+ED / RGB+D) used for the median depth and distortion.
 * Outputs colors [C,H,W,D], alphas [C,H,W,1], normals [C,H,W,3],
 * distort [C,H,W,1], median [C,H,W,1], last_ids, median_ids [C,H,W].
 * ws (hgsr_raster2d_fwd_ws_bytes) receives the packed 128-B surfel records (and, for a
 * training pack, the gradient slots' prefix). */
size_t hgsr_raster2d_fwd_ws_bytes(int C, int N, int D);
int hgsr_raster2d_fwd(int C, int N, int D, const float* means2d, const float* ray_transforms,
                      const float* colors, const float* opacities, const float* normals,
                      const float* backgrounds, int width, int height, int tile_size,
                      int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                      const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                      float* render_normals, float* render_distort, float* render_median,
                      int32_t* last_ids, int32_t* median_ids, void* ws, size_t ws_bytes,
                      hgsr_stream_t stream);
/* writes (overwrites) v_means2d [C*N,2], v_ray_transforms [C*N,9], v_colors [C*N,D],
 * v_opacities [C*N], v_normals [C*N,3], v_densify [C*N,2] (d loss / d screen
 * translation; nullable).  Deterministic gradient slots as hgsr_raster3d_bwd; ws:
 * hgsr_raster2d_bwd_ws_bytes(C, N, D, n_isects, fwd_ws != NULL). */
size_t hgsr_raster2d_bwd_ws_bytes(int C, int N, int D, int64_t n_isects, int reuse_fwd);
int hgsr_raster2d_bwd(int C, int N, int D, const float* means2d, const float* ray_transforms,
                      const float* colors, const float* opacities, const float* normals,
                      const float* backgrounds, int width, int height, int tile_size,
                      int tile_w, int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                      const int32_t* flatten_ids, const float* render_alphas,
                      const int32_t* last_ids, const float* v_render_colors,
                      const float* v_render_alphas, const float* v_render_normals,
                      float* v_means2d, float* v_ray_transforms, float* v_colors,
                      float* v_opacities, float* v_normals, float* v_densify,
                      const void* fwd_ws, void* ws, size_t ws_bytes, hgsr_stream_t stream);

/* Fused channel assembly for rasterization_2dgs (same conventions as
 * hgsr_raster3d_fwd_fused; the depth channel, when present, also drives the
 * median depth and the distortion map). */
int hgsr_raster2d_fwd_fused(int C, int N, int Dc, const float* means2d, const float* ray_transforms,
                            const float* colors, int colors_shared, const float* depths,
                            int expected_depth, const float* opacities, int opacities_shared,
                            const float* normals, const float* backgrounds, int width, int height,
                            int tile_size, int tile_w, int tile_h, const int32_t* isect_offsets,
                            int64_t n_isects, const int32_t* flatten_ids, float* render_colors,
                            float* render_alphas, float* render_normals, float* render_distort,
                            float* render_median, int32_t* last_ids, int32_t* median_ids, void* ws,
                            size_t ws_bytes, hgsr_stream_t stream);
/* hgsr_raster2d_fwd_fused split in two (as hgsr_raster3d_pack_fused / _fwd_packed): the
 * surfel records (ws, hgsr_raster2d_fwd_ws_bytes) are packed while the host reads the
 * intersection count, then composited; they stay valid as hgsr_raster2d_bwd_fused's fwd_ws.
 * qmask (nullable; size hgsr_raster3d_qmask_bytes, the same layout): the forward's
 * per-quadrant culling bits, read by hgsr_raster2d_bwd_fused instead of repeating the tests.
 * bwd_ws / ws_zeroed / isect_info: as hgsr_raster3d_fwd_packed (size
 * hgsr_raster2d_bwd_ws_bytes(C, N, D, n_isects, 1)).
 * normal_rot (nullable, the viewmats [C,4,4]): render_normals are written in world frame,
 * R^T n (rasterization_2dgs' frame), and hgsr_raster2d_bwd_fused given the same matrices
 * takes world-frame v_render_normals.  v_depth_extra (nullable, [C,H,W]): a second gradient
 * of the depth channel (K13's, the normals from the rendered depth), added per pixel by the
 * backward kernel instead of by a separate sum. */
/* radii (nullable, with the tile grid) and tiles_per_gauss (nullable): the records carry their
 * gradient slots, as hgsr_raster3d_pack_fused's (hgsr_raster2d_bwd_fused then gets fwd_slots = 1). */
int hgsr_raster2d_pack_fused(int C, int N, int Dc, const float* means2d, const float* ray_transforms,
                             const float* colors, int colors_shared, const float* depths,
                             const float* opacities, int opacities_shared, const float* normals,
                             const int32_t* radii, const int32_t* tiles_per_gauss, int tile_size, int tile_w,
                             int tile_h, void* ws, size_t ws_bytes, hgsr_stream_t stream);
int hgsr_raster2d_fwd_packed(int C, int N, int Dc, int with_depth, int expected_depth,
                             const float* backgrounds, int width, int height, int tile_size, int tile_w,
                             int tile_h, const int32_t* isect_offsets, int64_t n_isects,
                             const int32_t* flatten_ids, float* render_colors, float* render_alphas,
                             float* render_normals, float* render_distort, float* render_median,
                             int32_t* last_ids, int32_t* median_ids, const void* records,
                             size_t records_bytes, void* qmask, size_t qmask_bytes, void* bwd_ws,
                             size_t bwd_ws_bytes, const int64_t* isect_info, const float* normal_rot,
                             hgsr_stream_t stream);
int hgsr_raster2d_bwd_fused(int C, int N, int Dc, const float* means2d, const float* ray_transforms,
                            const float* colors, int colors_shared, const float* depths,
                            int expected_depth, const float* opacities, int opacities_shared,
                            const float* normals, const float* backgrounds, int width, int height,
                            int tile_size, int tile_w, int tile_h, const int32_t* isect_offsets,
                            int64_t n_isects, const int32_t* flatten_ids, const float* render_colors,
                            const float* render_alphas, const int32_t* last_ids,
                            const float* v_render_colors, const float* v_render_alphas,
                            const float* v_render_normals, float* v_means2d, float* v_ray_transforms,
                            float* v_colors, float* v_depths, float* v_opacities, float* v_normals,
                            float* v_densify, const void* fwd_ws, void* ws, size_t ws_bytes,
                            const void* qmask, size_t qmask_bytes, int ws_zeroed,
                            const float* normal_rot, const float* v_depth_extra, const int32_t* radii,
                            int fwd_slots, hgsr_stream_t stream);

/* ---- K14: anchor -> neural-Gaussian decode --------------
 * replaces scene/lod_model.py:286-290 set_anchor_mask (LoD mask, dist2level
 * 'floor') and scene/basic_model.py:297-371 generate_neural_gaussians with the MLPs
 * of scene/lod_model.py:67-84 (appearance_dim = 0, smooth_complement = 1).
 * mask[A] = level <= clamp(floor(log2(sd / (|anchor - cam| * res_scale)) / log2_fork
 * + extra_level), 0, max_level); cam_center is a device pointer to 3 floats. */
int hgsr_lod_mask(int A, const float* anchor, const int32_t* level, const float* extra_level,
                  const float* cam_center, float res_scale, float standard_dist, float log2_fork,
                  int max_level, uint8_t* mask, hgsr_stream_t stream);
/* Decode of Av visible anchors (vis_idx [Av] int32 anchor ids, NULL = 0..Av-1):
 * feat_dim F = 32, view_dim 0 or 3, n_offsets <= 11, color_dim = 3 (RGB) or
 * 3 (deg+1)^2 (SH); mlp is a HOST array of 12 device pointers: for the opacity,
 * cov and colour heads in that order {w1 [F, F+vd], b1 [F], w2 [O, F], b2 [O]}
 * (nn.Linear layout).  Two passes: hgsr_decode_count writes the number of kept
 * Gaussians (tanh opacity > 0) to *total (device int64), the caller sizes the
 * outputs, hgsr_decode_fwd writes them in the reference order (anchor-major, then
 * offset): xyz, offsets (scaled), color [M, cd], opacity [M], scaling [M,3],
 * rot [M,4]; mask [Av*n_offsets] (uint8) and slot_row [Av*n_offsets] (output row
 * or -1, consumed by the backward).  ws: hgsr_decode_ws_bytes(Av), kept between
 * the two calls.  av_dev (nullable, device int64): the visible count is read on the
 * device (as hgsr_explicit_count wrote it) and the count pass's Av is only its upper
 * bound (the workspace is sized for it) -- the prefilter then needs no host read; the
 * caller reads *av_dev together with *total and passes the real Av to hgsr_decode_fwd. */
size_t hgsr_decode_ws_bytes(int Av);
int hgsr_decode_count(int Av, int F, int view_dim, int n_offsets, int color_dim,
                      const int32_t* vis_idx, const float* anchor, const float* feat,
                      const float* cam_center, const float* const* mlp, void* ws, size_t ws_bytes,
                      int64_t* total, const int64_t* av_dev, hgsr_stream_t stream);
int hgsr_decode_fwd(int Av, int F, int view_dim, int n_offsets, int color_dim,
                    const int32_t* vis_idx, const float* anchor, const float* feat,
                    const float* offset, const float* scaling_raw, const float* cam_center,
                    const float* const* mlp, float* xyz, float* offsets_out, float* color,
                    float* opacity, float* scaling, float* rot, uint8_t* mask, int32_t* slot_row,
                    void* ws, size_t ws_bytes, hgsr_stream_t stream);

/* vjp of the decode.  Gradients of the outputs (rows as written by
 * hgsr_decode_fwd; any of them may be NULL = zero): g_xyz, g_offsets, g_color,
 * g_opacity, g_scaling, g_rot.  Results are ACCUMULATED (+=) into caller-zeroed
 * d_anchor [A,3] (nullable), d_feat [A,F], d_scaling [A,6] (d w.r.t. the raw
 * _scaling parameter) and the 12 weight gradients d_mlp (same order as mlp);
 * d_offset [A, n_offsets, 3] rows of visible anchors are written.  Weight
 * gradients are reduced in a fixed order (deterministic; the launch grids are fixed by the
 * compiled code, not the device, so the bits are the same on every MI355X).
 * head_mask (bit 0 opacity, 1 cov, 2 colour; 0 = all): the heads this call runs, cov first.
 * After the cov head d_offset, d_scaling and the cov weights are final: a data-parallel
 * caller runs {cov}, launches their all-reduce, then {opacity, colour} (the other
 * accumulations continue).  ws: hgsr_decode_bwd_ws_bytes(Av). */
size_t hgsr_decode_bwd_ws_bytes(int Av);
/* the SH colour head's backward form for later hgsr_decode_bwd calls: 1 (default) one launch,
 * 0 the chunked launches (the tests compare both); -1 only queries.  Returns the previous form. */
int hgsr_decode_set_color_bwd(int one);
int hgsr_decode_bwd(int Av, int F, int view_dim, int n_offsets, int color_dim,
                    const int32_t* vis_idx, const float* anchor, const float* feat,
                    const float* offset, const float* scaling_raw, const float* cam_center,
                    const float* const* mlp, const int32_t* slot_row, const float* g_xyz,
                    const float* g_offsets, const float* g_color, const float* g_opacity,
                    const float* g_scaling, const float* g_rot, float* d_anchor, float* d_feat,
                    float* d_offset, float* d_scaling, float* const* d_mlp, int head_mask,
                    void* ws, size_t ws_bytes, hgsr_stream_t stream);

/* ---- K13: normals from the rendered depth (2DGS) -------------------------------
 * replaces the gsplat fork's depth_to_normal (torch, ~25 launches incl. two 3 x 3 x HW GEMMs
 * per direction) used by rasterization_2dgs for render_normals_from_depth (reference
 * gaussian_renderer/render.py:62-76; consumed by train.py:180-188).  depth [C,H,W] with
 * strides depth_strides (elements; e.g. the expected-depth channel of render_colors),
 * camtoworlds [C,4,4], Ks [C,3,3]; z_depth = 0 normalises the ray directions.  normals
 * [C,H,W,3] (written; 0 on the one-pixel border).  The backward writes v_depth [C,H,W]
 * (contiguous) from v_normals [C,H,W,3]; no gradient to the cameras.  from_viewmat = 1: the
 * [C,4,4] matrices are world -> camera viewmats (the rotation is transposed in place). */
int hgsr_depth_normal_fwd(int C, int H, int W, const float* depth, const int64_t* depth_strides,
                          const float* camtoworlds, const float* Ks, int z_depth, int from_viewmat,
                          float* normals, hgsr_stream_t stream);
int hgsr_depth_normal_bwd(int C, int H, int W, const float* depth, const int64_t* depth_strides,
                          const float* camtoworlds, const float* Ks, int z_depth, int from_viewmat,
                          const float* v_normals, float* v_depth, hgsr_stream_t stream);
/* out[c,m] = R_c in[c,m] (transpose = 0) or R_c^T in[c,m] (transpose = 1), 3-vectors; R_c is
 * the 3x3 block at R + c*cam_stride with rows row_stride floats apart (9/3 for [C,3,3], 16/4
 * for the rotation block of [C,4,4] viewmats): rasterization_2dgs's camera -> world rotation of
 * render_normals (an einsum the fork runs as a 3 x 3 x HW GEMM) and its vjp. */
int hgsr_rotate3(int C, int64_t M, const float* R, int cam_stride, int row_stride, int transpose,
                 const float* in, float* out, hgsr_stream_t stream);

/* ---- K15: fused training loss ---------------------------
 * replaces the loss head of reference train.py:153-202 with utils/loss_utils.py:17-60:
 * x = image*mask, y = gt*mask (image, gt [C,H,W], C <= 3; mask [H,W] nullable); out[9] (device) =
 * {loss, l1, ssim, sky, entropy, scale_reg, normal, distortion, inv_depth} with
 *   loss = (1-l)*mean|x-y| + l*(1-mean SSIM(x,y)) + l_dreg*mean_i prod_j scaling[i,j]
 *        + l_sky*mean(-(1-mask) log(1-a)) + l_ent*mean(-a log a)       (a = clamp(alpha, 1e-6, 1-1e-6))
 *        + l_normal*mean((1 - sum_c n_c nfd_c alpha) * mask)          (train.py:180-188, alpha detached)
 *        + l_dist*mean(distort * mask)                                  (train.py:190-191)
 *        + l_depth*mean(|(invD - mono) * depth_mask|), invD = depth > 0 ? 1/depth : 0  (train.py:193-199)
 * (alpha [H,W] nullable when both l_sky and l_ent are 0; scaling [n_scaling, k_scaling]
 * contiguous, nullable, scale_reg = 0 when n_scaling = 0 as train.py:163-166; the aux
 * inputs are nullable and their terms 0 when absent).
 * ws (hgsr_loss_ws_bytes) holds the SSIM derivative maps for hgsr_loss_bwd, which writes
 * g_image, g_alpha [H,W] (nullable), g_scaling (nullable) and the aux gradients
 * (nullable) from g_outs[9] (host array of device pointers to the upstream gradients of the
 * nine 0-dim outputs; a NULL entry is a zero gradient).
 * *_strides (host, nullable / zero = contiguous): element strides {channel, row, column}
 * ({row, column} for [H,W] maps), e.g. {1, 3W, 3} for the channels-last render output
 * seen through permute(2,0,1) (render.py:81-95); every gradient is written with its
 * input's strides.  g_image channels C..C+extra_channels-1 (trailing render channels the
 * loss ignores, e.g. the depth of RGB+ED) are written as zero. */
typedef struct hgsr_loss_terms {
    float lambda_dssim, lambda_sky_opa, lambda_entropy, lambda_dreg;
    float lambda_normal, lambda_dist, lambda_depth;
    const float* normals;            /* render_normals [3,H,W] view */
    int64_t normals_strides[3];
    const float* normals_from_depth; /* render_normals_from_depth [3,H,W] view */
    int64_t nfd_strides[3];
    const float* distort;            /* render_distort [H,W] view */
    int64_t distort_strides[2];
    const float* depth;              /* render_depth [H,W] view */
    int64_t depth_strides[2];
    const float* mono_invdepth;      /* [H,W] contiguous */
    const float* depth_mask;         /* [H,W] contiguous, nullable */
} hgsr_loss_terms;
typedef struct hgsr_loss_aux_grads {
    float* g_normals;
    float* g_normals_from_depth;
    float* g_distort;
    float* g_depth;
} hgsr_loss_aux_grads;
size_t hgsr_loss_ws_bytes(int C, int H, int W);
int hgsr_loss_fwd(int C, int H, int W, const float* image, const int64_t* image_strides,
                  const float* gt, const int64_t* gt_strides, const float* mask, const float* alpha,
                  const float* scaling, int64_t n_scaling, int k_scaling, const hgsr_loss_terms* terms,
                  float* out, void* ws, size_t ws_bytes, hgsr_stream_t stream);
int hgsr_loss_bwd(int C, int H, int W, const float* image, const int64_t* image_strides,
                  const float* gt, const int64_t* gt_strides, const float* mask, const float* alpha,
                  const float* scaling, int64_t n_scaling, int k_scaling, const hgsr_loss_terms* terms,
                  const float* const* g_outs, float* g_image, int extra_channels, float* g_alpha,
                  float* g_scaling, const hgsr_loss_aux_grads* aux_grads, const void* ws,
                  size_t ws_bytes, hgsr_stream_t stream);

/* ---- K16: densification on device ----------------------
 * hgsr_training_statis replaces BasicModel.training_statis (scene/basic_model.py:96-144):
 * vis_idx [Av] = nonzero(visible_mask) (ascending); selection [Av*n_offsets] = the decode's
 * opacity > 0 mask; selection_rank [Av*n_offsets] its exclusive prefix (= output row);
 * visibility_filter [M] (radii > 0), viewspace_grad [M,2] (means2d.grad), opacity [M],
 * radii [M] (max growing only) for the M decoded Gaussians.  Updates in place (float32):
 * anchor_opacity_accum / anchor_demon [A], offset_gradient_accum / offset_denom /
 * max_radii2D / offset_opacity_accum [A*n_offsets] ("mean" or "max" pruning / growing
 * types; the reference scales the gradient by (W/2, H/2) before the norm).
 * One lane per visible anchor, slots in order (n_offsets <= 16): deterministic. */
int hgsr_training_statis(int Av, int n_offsets, int width, int height, int pruning_max, int growing_max,
                         const int32_t* vis_idx, const uint8_t* selection, const int32_t* selection_rank,
                         const uint8_t* visibility_filter, const float* viewspace_grad,
                         const float* opacity, const int32_t* radii, float* anchor_opacity_accum,
                         float* anchor_demon, float* offset_gradient_accum, float* offset_denom,
                         float* max_radii2D, float* offset_opacity_accum, hgsr_stream_t stream);
/* replaces get_remove_duplicates (scene/basic_model.py:179-190): found[i] = 1 iff
 * cand_coords[i] (int32 xyz voxel) equals some grid_coords row.  Hash set in ws
 * (hgsr_voxel_dedup_ws_bytes); coordinates must lie in [-(2^20-1), 2^20-1] (bit 0 of
 * *overflow, device int32, is set otherwise). */
size_t hgsr_voxel_dedup_ws_bytes(int64_t n_grid);
int hgsr_voxel_dedup(int64_t n_grid, const int32_t* grid_coords, int64_t n_cand, const int32_t* cand_coords,
                     uint8_t* found, int32_t* overflow, void* ws, size_t ws_bytes, hgsr_stream_t stream);
/* torch_scatter.scatter_max(src [n,F], index [n] int64, dim=0, dim_size=n_out)[0]
 * (scene/lod_model.py:559): out [n_out,F]; rows no index reaches are 0. */
int hgsr_scatter_max(int64_t n, int F, const float* src, const int64_t* index, int64_t n_out, float* out,
                     hgsr_stream_t stream);
/* GaussianLoDModel.weed_out (scene/lod_model.py:236-249, weed_ratio > 0 branch):
 * mask[i] = mean over cameras (cam_infos [n_cams,4] = centre xyz, resolution scale) of
 * levels[i] <= map_to_int_level(log2(standard_dist / dist) / log2(fork), street_levels-1)
 * > weed_ratio.  dist2level_mode: 0 floor, 1 round, 2 ceil, 3 progressive. */
int hgsr_weed_out(int64_t n, const float* positions, const int32_t* levels, int n_cams,
                  const float* cam_infos, float standard_dist, float fork, int street_levels,
                  int dist2level_mode, float weed_ratio, uint8_t* mask, hgsr_stream_t stream);

/* ---- K17: optimizer step ------------------------------------------------------
 * replaces gaussians.optimizer.step() (reference train.py:274-277) of
 * torch.optim.Adam(l, lr=0.0, eps=1e-15) (scene/lod_model.py:320; per-group lr from
 * update_learning_rate, scene/lod_model.py:350-372), all parameters in one launch
 * (chunks of 16 tensors).  Per tensor: param / grad / exp_avg / exp_avg_sq device
 * pointers (fp32, numel elements each, updated in place), its group's lr and its
 * 1-based step count (torch's per-parameter state["step"] after the increment).
 * grad == NULL skips the tensor (torch skips parameters whose .grad is None).
 * amsgrad, weight_decay and maximize are not used by the reference and not offered. */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    double lr;
    int64_t step;
} hgsr_adam_tensor;
int hgsr_adam_step(int n_tensors, const hgsr_adam_tensor* tensors, double beta1, double beta2, double eps,
                   hgsr_stream_t stream);

/* ---- explicit (merged-scene) Gaussians: the c5 render path -------------------
 * Reference render() with pc.explicit_gs (gaussian_renderer/render.py:22-25):
 * set_gs_mask (scene/lod_model.py:292-296) + generate_explicit_gaussians
 * (scene/basic_model.py:373-383) as one ordered stream compaction.
 * hgsr_explicit_count: with visible == NULL, the LoD mask of the N centres (same test as
 * hgsr_lod_mask) is written to mask[N] (bytes); otherwise `visible` [N] bytes is used as the
 * mask.  Writes the kept count to *total (device int64) and the block bases to ws
 * (hgsr_explicit_ws_bytes(N)), which hgsr_explicit_gather / _scatter read. */
size_t hgsr_explicit_ws_bytes(int64_t N);
int hgsr_explicit_count(int64_t N, const float* xyz, const int32_t* level, const float* extra_level,
                        const float* cam_center, float res_scale, float standard_dist, float log2_fork,
                        int max_level, const uint8_t* visible, uint8_t* mask, void* ws, size_t ws_bytes,
                        int64_t* total, hgsr_stream_t stream);
/* kept rows in source order: out_xyz [M,3], out_color [M,K,3] = cat(f_dc [N,1,3],
 * f_rest [N,K-1,3]) rows, out_opacity [M,1], out_scaling [M,3], out_rotation [M,4],
 * out_index [M] (source row).  M = the count of hgsr_explicit_count. */
int hgsr_explicit_gather(int64_t N, int K, const uint8_t* mask, const float* xyz, const float* f_dc,
                         const float* f_rest, const float* opacity, const float* scaling, const float* rotation,
                         const void* ws, size_t ws_bytes, float* out_xyz, float* out_color, float* out_opacity,
                         float* out_scaling, float* out_rotation, int32_t* out_index, hgsr_stream_t stream);
/* vjp of the gather: every source row's gradient (OVERWRITTEN) is its output row's gradient,
 * or 0 where the mask dropped it; any g_* / v_* may be NULL (g NULL = zero). */
int hgsr_explicit_scatter(int64_t N, int K, const uint8_t* mask, const void* ws, size_t ws_bytes,
                          const float* g_xyz, const float* g_color, const float* g_opacity, const float* g_scaling,
                          const float* g_rotation, float* v_xyz, float* v_f_dc, float* v_f_rest, float* v_opacity,
                          float* v_scaling, float* v_rotation, hgsr_stream_t stream);

/* Ordered indices of the set bytes of mask[N] into index[M] (M = the count written by
 * hgsr_explicit_count(visible = mask) into the same ws). */
int hgsr_mask_index(int64_t N, const uint8_t* mask, const void* ws, size_t ws_bytes, int32_t* index,
                    hgsr_stream_t stream);
/* Anchor prefilter (reference gaussian_renderer/render.py:120-197 prefilter_voxel, after
 * set_anchor_mask scene/lod_model.py:286-290): visible[a] = 1 iff the LoD test passes (when
 * level != NULL; the test of hgsr_lod_mask) and the anchor projected with scales[a*stride .. +3]
 * (activated) and quats[a] by camera (viewmat [4,4], K [3,3]) has radius > 0, with the
 * projection of hgsr_project3d_fwd (same bits).  Writes no projection outputs. */
int hgsr_anchor_prefilter(int A, const float* anchor, const float* quats, const float* scales, int scale_stride,
                          const float* viewmat, const float* K, int width, int height, float eps2d,
                          float near_plane, float far_plane, const int32_t* level, const float* extra_level,
                          const float* cam_center, float res_scale, float standard_dist, float log2_fork,
                          int max_level, uint8_t* visible, hgsr_stream_t stream);

/* ---- 3DGS parametrisation activations of a train step (scaling_activation = exp,
 * opacity_activation = sigmoid of the reference models): scales [N,3] = exp(log_scales),
 * opacities [N] = sigmoid(logits) in one pass; the vjp writes (OVERWRITES) v_log_scales =
 * v_scales * scales and v_logits = v_opacities * o (1 - o) (either output nullable; a NULL
 * upstream gradient counts as zero). */
int hgsr_activate_fwd(int64_t N, const float* log_scales, const float* logits, float* scales, float* opacities,
                      hgsr_stream_t stream);
int hgsr_activate_bwd(int64_t N, const float* scales, const float* opacities, const float* v_scales,
                      const float* v_opacities, float* v_log_scales, float* v_logits, hgsr_stream_t stream);

/* ---- measurement ----------------------------------------------------------
 * Optional per-kernel HIP-event timing used by bench.py (roofline numbers):
 * when enabled, the main kernel of every entry point is bracketed by
 * hipEventRecord on the stream it is launched on.  Not for production use
 * (events are pooled; at most 1<<16 records between resets). */
int hgsr_timing_enable(int on);
int hgsr_timing_reset(void);
/* restrict the recording to one kernel name (NULL = every kernel): bench.py times only
 * the dominant kernel inside its timed region, so the events add no per-launch overhead
 * to the other kernels of the step. */
int hgsr_timing_only(const char* kernel);
/* (pixel, Gaussian) pairs the timed raster backward visited (every Gaussian up to each tile's
 * latest contributor x 256 pixels), counted on the device while raster3d_bwd / raster2d_bwd
 * is being timed; synchronises the device; reset = 1 zeroes the counter. */
int hgsr_timing_pairs(unsigned long long* out, int reset);
/* lane-pairs the timed raster backward actually stepped: every entry of each wave's
 * compacted per-batch list (Gaussians whose footprint reaches the wave's 8x8 quadrant)
 * x 64 lanes, counted with the pairs above (read before a resetting hgsr_timing_pairs). */
int hgsr_timing_exec_pairs(unsigned long long* out);
/* total milliseconds and launch count recorded for `kernel` (synchronises the
 * recorded events); kernel names: project3d_fwd, project3d_bwd, project2d_fwd,
 * project2d_bwd, sh_fwd, sh_bwd, isect_count, isect_emit, tile_sort,
 * raster3d_fwd, raster3d_bwd, raster2d_fwd, raster2d_bwd. */
int hgsr_timing_query(const char* kernel, double* total_ms, int64_t* count);

#ifdef __cplusplus
}
#endif
#endif /* HGSR_H */
