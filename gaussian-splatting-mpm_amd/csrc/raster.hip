// raster.hip -- 3D Gaussian splatting forward for MI355X (gfx950).
//
// Drop-in for diff_gaussian_rasterization._C.rasterize_gaussians (forward), the
// third-party CUDA extension the reference calls at main.py:148-156 (pre-2024
// API: returns color [3,H,W] and radii [P]).  Pipeline:
//
//   k_preprocess   one lane per Gaussian: frustum test (view z > 0.2), EWA 2D
//                  covariance (+0.3 low-pass), conic, 3-sigma radius, 16x16
//                  tile rect, SH(deg<=3) -> RGB, depth, tiles touched
//   scan           inclusive sum of tiles touched (rocPRIM) -> K, one D2H
//   depth order    stable sort of the P depths (ties keep index order), then
//                  the tiles-touched counts scanned in that order; queued
//                  before the K read-back, so they run behind the simulator
//   k_emit_pairs   each (Gaussian, tile) pair, in depth order, written at
//                  its depth-order offset (one lane per pair)
//   sort           stable onesweep radix sort on the tile index alone
//                  (msb(#tiles) bits): each tile's list comes out in (depth,
//                  index) order, the list upstream's 64-bit
//                  (tile << 32 | depth bits) sort produces
//                  (GSMPM_RASTER_WIDE_KEYS=1 runs that upstream path instead)
//   k_ranges32     per-tile [start, end) in the sorted list
//   k_render       one wave64 per 8x8 quarter of a 16x16 tile; batches of 64
//                  list entries are culled against the sub-tile (alpha can't
//                  reach 1/255 there -> dropped, exactly the entries the blend
//                  would skip), compacted in LDS and blended front to back
//                  with the upstream cut-offs (alpha < 1/255 skip, alpha <=
//                  0.99, T < 1e-4 stop), wave early exit; records each
//                  pixel's final T and last contributor for the backward.
//
// Backward (upstream's BACKWARD::render + preprocess, for extra.py's
// training loop):
//   k_render_bwd     one workgroup per tile, back to front from each pixel's
//                    last contributor; the 256 pixels' contributions to each
//                    (Gaussian, tile) pair are summed on chip (wave shuffles +
//                    LDS) and stored once per pair at the pair's emission
//                    index in Gaussian-index order (k_slots derives it for
//                    the depth-ordered path), so a Gaussian's pairs are
//                    contiguous (no global atomics);
//   k_preprocess_bwd one lane per Gaussian: sums its pair records, then the
//                    2D-covariance / projection / SH / 3D-covariance adjoints.
#include <hip/hip_runtime.h>

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <chrono>
#include <cstdlib>
#include <mutex>
#include <atomic>
#include <vector>
#include <cstring>
#include <string>

#include "common.h"

namespace gsmpm {

constexpr int kBX = 16, kBY = 16, kBlock = kBX * kBY;
// rocPRIM's onesweep radix sort at every size above one block, for the tile
// sort (its default switches to block sort + merge passes below 1M keys: ~15
// launches instead of one per 8-bit digit; measured 0.05 ms/frame slower on the
// bench's ~500k pairs).  The 100k-key depth sort keeps the default: there the
// merge path is the faster one (onesweep's look-back chain dominates).
// GSMPM_OS_BLOCK / GSMPM_OS_ITEMS (A/B builds): an explicit onesweep block config instead of rocPRIM's
// default for the arch (gfx950 has no tuned entry and takes the generic 256 x 16, 8-bit digits).
#ifndef GSMPM_OS_BLOCK
#define GSMPM_OS_BLOCK 0
#endif
#ifndef GSMPM_OS_ITEMS
#define GSMPM_OS_ITEMS 16
#endif
#if GSMPM_OS_BLOCK > 0
using OnesweepSort = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<GSMPM_OS_BLOCK, GSMPM_OS_ITEMS>,
                                        rocprim::kernel_config<GSMPM_OS_BLOCK, GSMPM_OS_ITEMS>, 8,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
#else
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;
#endif
// The depth sort takes onesweep from this many Gaussians on (GSMPM_DEPTH_OS_MIN; below it rocPRIM's
// default block sort + merge passes, which win at lego's 100k keys); 0 = never.  Bicycle (1M): render
// 1.256 -> 1.241 ms (3 interleaved rounds, tools/ab_render_os.sh; explicit 512 / 1024 x 16 onesweep
// blocks for the tile sort measured 1.256 / 1.260 ms, so the tile sort keeps rocPRIM's default)
#ifndef GSMPM_DEPTH_OS_MIN
#define GSMPM_DEPTH_OS_MIN 262144
#endif
constexpr size_t kDepthOnesweepMin = GSMPM_DEPTH_OS_MIN;

__constant__ float kSH_C0 = 0.28209479177387814f;
__constant__ float kSH_C1 = 0.4886025119029199f;
__constant__ float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f, -1.0925484305920792f,
                                0.5462742152960396f};
__constant__ float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f, 0.3731763325901154f,
                                -0.4570457994644658f, 1.445305721320277f, -0.5900435899266435f};

struct RasterDev {
  int P, D, M, W, H;
  const float *means3D, *shs, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp;
  float scale_modifier;
  const float *viewmatrix, *projmatrix, *campos, *bg;
  float tanfovx, tanfovy, focal_x, focal_y;
  int grid_x, grid_y;
  int tight;  // bin each Gaussian into the tiles its alpha >= 1/255 box reaches (k_preprocess)
  int sh_vec4;  // M == 16 and shs 16-byte aligned: a Gaussian's 48 SH floats as 12 dwordx4 loads
};

__device__ __forceinline__ void xform4x3(const float* p, const float* m, float o[3]) {
  o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
  o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
  o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}

__device__ __forceinline__ float ndc2pix(float v, int S) { return ((v + 1.0f) * S - 1.0f) * 0.5f; }

__device__ __forceinline__ void get_rect(float px, float py, int r, int gx, int gy, int rmin[2], int rmax[2]) {
  rmin[0] = min(gx, max(0, (int)((px - r) / kBX)));
  rmin[1] = min(gy, max(0, (int)((py - r) / kBY)));
  rmax[0] = min(gx, max(0, (int)((px + r + kBX - 1) / kBX)));
  rmax[1] = min(gy, max(0, (int)((py + r + kBY - 1) / kBY)));
}

// a Gaussian's binning rect [x0, x1) x [y0, y1) in tiles, 16 bits each (k_preprocess writes it)
__device__ __forceinline__ uint2 pack_rect(int x0, int y0, int x1, int y1) {
  return make_uint2((unsigned)x0 | ((unsigned)y0 << 16), (unsigned)x1 | ((unsigned)y1 << 16));
}
__device__ __forceinline__ void unpack_rect(uint2 r, int rmin[2], int rmax[2]) {
  rmin[0] = (int)(r.x & 0xffffu);
  rmin[1] = (int)(r.x >> 16);
  rmax[0] = (int)(r.y & 0xffffu);
  rmax[1] = (int)(r.y >> 16);
}

// computeCov3D: Sigma = R diag(s*mod)^2 R^T, R from the (unnormalised) quaternion (r,x,y,z)
__device__ __forceinline__ void cov3d_from_sr(const float* s, float mod, const float* rot, float c6[6]) {
  const float S0 = mod * s[0], S1 = mod * s[1], S2 = mod * s[2];
  const float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
  const float R[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y)},
                         {2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x)},
                         {2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
  float M[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    M[i][0] = R[i][0] * S0;
    M[i][1] = R[i][1] * S1;
    M[i][2] = R[i][2] * S2;
  }
  float Sg[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Sg[i][j] = M[i][0] * M[j][0] + M[i][1] * M[j][1] + M[i][2] * M[j][2];
  c6[0] = Sg[0][0];
  c6[1] = Sg[0][1];
  c6[2] = Sg[0][2];
  c6[3] = Sg[1][1];
  c6[4] = Sg[1][2];
  c6[5] = Sg[2][2];
}

// computeCov2D: EWA projection J W Vrk W^T J^T with the 1.3 x fov clamp and +0.3 low-pass
__device__ __forceinline__ void cov2d(const float* mean, const RasterDev& a, const float* c3, float out[3]) {
  float t[3];
  xform4x3(mean, a.viewmatrix, t);
  const float limx = 1.3f * a.tanfovx, limy = 1.3f * a.tanfovy;
  const float txtz = t[0] / t[2], tytz = t[1] / t[2];
  t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
  t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
  const float J00 = a.focal_x / t[2], J02 = -(a.focal_x * t[0]) / (t[2] * t[2]);
  const float J11 = a.focal_y / t[2], J12 = -(a.focal_y * t[1]) / (t[2] * t[2]);
  const float* vm = a.viewmatrix;
  const float W[3][3] = {{vm[0], vm[4], vm[8]}, {vm[1], vm[5], vm[9]}, {vm[2], vm[6], vm[10]}};
  float T[2][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    T[0][c] = J00 * W[0][c] + J02 * W[2][c];
    T[1][c] = J11 * W[1][c] + J12 * W[2][c];
  }
  const float V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
  float TV[2][3];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) TV[r][c] = T[r][0] * V[0][c] + T[r][1] * V[1][c] + T[r][2] * V[2][c];
  const float ca = TV[0][0] * T[0][0] + TV[0][1] * T[0][1] + TV[0][2] * T[0][2];
  const float cb = TV[0][0] * T[1][0] + TV[0][1] * T[1][1] + TV[0][2] * T[1][2];
  const float cc = TV[1][0] * T[1][0] + TV[1][1] * T[1][1] + TV[1][2] * T[1][2];
  out[0] = ca + 0.3f;
  out[1] = cb;
  out[2] = cc + 0.3f;
}

// VEC4: the Gaussian's 48 coefficients arrive as 12 16-byte loads into
// registers (one lane's 192 B are contiguous; 48 scalar loads made every load
// instruction touch 64 cache lines); the arithmetic is the same either way
template <bool VEC4>
__device__ __forceinline__ void sh_rgb(const RasterDev& a, int idx, const float* pos, float rgb[3], unsigned& clamp) {
  float dir[3] = {pos[0] - a.campos[0], pos[1] - a.campos[1], pos[2] - a.campos[2]};
  const float len = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
  dir[0] /= len;
  dir[1] /= len;
  dir[2] /= len;
  const float* shg = a.shs + (size_t)idx * a.M * 3;
  float shv[VEC4 ? 48 : 1];
  if constexpr (VEC4) {
    const float4* s4 = reinterpret_cast<const float4*>(shg);
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      const float4 v = s4[q];
      shv[4 * q] = v.x;
      shv[4 * q + 1] = v.y;
      shv[4 * q + 2] = v.z;
      shv[4 * q + 3] = v.w;
    }
  }
  const float* sh = VEC4 ? shv : shg;
  const float x = dir[0], y = dir[1], z = dir[2];
  const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float r = kSH_C0 * sh[0 * 3 + ch];
    if (a.D > 0) {
      r = r - kSH_C1 * y * sh[1 * 3 + ch] + kSH_C1 * z * sh[2 * 3 + ch] - kSH_C1 * x * sh[3 * 3 + ch];
      if (a.D > 1) {
        r = r + kSH_C2[0] * xy * sh[4 * 3 + ch] + kSH_C2[1] * yz * sh[5 * 3 + ch] +
            kSH_C2[2] * (2.0f * zz - xx - yy) * sh[6 * 3 + ch] + kSH_C2[3] * xz * sh[7 * 3 + ch] +
            kSH_C2[4] * (xx - yy) * sh[8 * 3 + ch];
        if (a.D > 2) {
          r = r + kSH_C3[0] * y * (3.0f * xx - yy) * sh[9 * 3 + ch] + kSH_C3[1] * xy * z * sh[10 * 3 + ch] +
              kSH_C3[2] * y * (4.0f * zz - xx - yy) * sh[11 * 3 + ch] +
              kSH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12 * 3 + ch] +
              kSH_C3[4] * x * (4.0f * zz - xx - yy) * sh[13 * 3 + ch] + kSH_C3[5] * z * (xx - yy) * sh[14 * 3 + ch] +
              kSH_C3[6] * x * (xx - 3.0f * yy) * sh[15 * 3 + ch];
        }
      }
    }
    r += 0.5f;
    clamp |= (r < 0.0f ? 1u : 0u) << ch;
    rgb[ch] = fmaxf(r, 0.0f);
  }
}

constexpr int kSub = 8;  // pixel sub-tile side: one wave of pixels

// can alpha = o exp(power) reach 1/255 at a pixel centre of the sub-tile
// [x0, x0 + 7] x [y0, y0 + 7]?  Conservative; NaNs keep the Gaussian.  The
// Gaussian-only part (the ellipse's half extents) is factored out so the
// emission computes it once per Gaussian, not once per (tile, quarter).
struct Reach {
  float ex, ey;  // half extents of the alpha >= 1/255 ellipse's box, + 1 px
  int mode;      // 0: test the box, 1: reaches nothing (o < 1/255), 2: keep (degenerate conic)
};
__device__ __forceinline__ Reach reach_of(float4 co) {
  Reach r{0.f, 0.f, 0};
  if (co.w * 255.0f < 0.999f) {  // o < 1/255: alpha < 1/255 everywhere
    r.mode = 1;
    return r;
  }
  const float det = co.x * co.z - co.y * co.y;
  if (!(det > 0.0f)) {
    r.mode = 2;
    return r;
  }
  const float k = fmaxf(2.0f * __logf(255.0f * co.w), 0.0f) * 1.02f + 0.02f;
  r.ex = sqrtf(k * co.z / det) + 1.0f;
  r.ey = sqrtf(k * co.x / det) + 1.0f;
  return r;
}
__device__ __forceinline__ bool reaches_box(const Reach& r, float2 g, float x0, float y0) {
  if (r.mode) return r.mode == 2;
  return !(g.x + r.ex < x0 || g.x - r.ex > x0 + (kSub - 1) || g.y + r.ey < y0 || g.y - r.ey > y0 + (kSub - 1));
}
__device__ __forceinline__ bool reaches_subtile(float2 g, float4 co, float x0, float y0) {
  return reaches_box(reach_of(co), g, x0, y0);
}

// Tight binning (RasterDev::tight).  A (Gaussian, tile) pair whose four
// sub-tiles the Gaussian's alpha-reach box misses is one upstream's blend
// skips at every pixel of the tile.  The box is axis-aligned, so the tiles it
// reaches within the 3-sigma rect are themselves a rect: the sub-tile columns
// c (pixels [8c, 8c + 7]) that reaches_box passes are those with
// !(lo > 8c + 7) (true from some c on) and !(hi < 8c) (true up to some c),
// an interval, and likewise for rows.  k_preprocess bins the Gaussian into
// that rect only, with reaches_box's own comparisons on the same floats, so
// every emitted pair reaches at least one sub-tile and no pair that reaches
// one is lost: the tile lists are the culled lists k_render walks, and K
// shrinks before the sort.  num_rendered stays upstream's 3-sigma count.
// [first, last] sub-cells of [c0, c1) the box [lo, hi] reaches (first > last: none)
__device__ __forceinline__ void reach_cells(float lo, float hi, int c0, int c1, int& first, int& last) {
  int a = c0, b = c1;
  while (a < b) {  // first c with !(lo > 8c + 7)
    const int m = (a + b) >> 1;
    if (!(lo > (float)(m * kSub) + (kSub - 1))) b = m;
    else a = m + 1;
  }
  first = a;
  a = c0;
  b = c1;
  while (a < b) {  // first c with hi < 8c
    const int m = (a + b) >> 1;
    if (hi < (float)(m * kSub)) b = m;
    else a = m + 1;
  }
  last = a - 1;
}

#include "scan.h"
#include "dsort.h"
#include "lsd.h"

// returns the depth bits of a visible Gaussian (tiles word != 0), else 0
__device__ __forceinline__ unsigned preprocess_one(const RasterDev& a, int idx, int* __restrict__ radii,
                                                   float* __restrict__ depth, float2* __restrict__ xy,
                                                   float4* __restrict__ conic_o, float4* __restrict__ rgbo,
                                                   unsigned long long* __restrict__ tiles, uint2* __restrict__ rect) {
  radii[idx] = 0;
  tiles[idx] = 0;  // (3-sigma tile count << 32) | binned tile count
  const float* p = a.means3D + (size_t)idx * 3;
  float pv[3];
  xform4x3(p, a.viewmatrix, pv);
  if (pv[2] <= 0.2f) return 0u;
  const float* pm = a.projmatrix;
  const float hx = pm[0] * p[0] + pm[4] * p[1] + pm[8] * p[2] + pm[12];
  const float hy = pm[1] * p[0] + pm[5] * p[1] + pm[9] * p[2] + pm[13];
  const float hw = pm[3] * p[0] + pm[7] * p[1] + pm[11] * p[2] + pm[15];
  const float pw = 1.0f / (hw + 0.0000001f);
  const float ppx = hx * pw, ppy = hy * pw;
  float c6[6];
  const float* c3;
  if (a.cov3D_precomp) {
    c3 = a.cov3D_precomp + (size_t)idx * 6;
  } else {
    cov3d_from_sr(a.scales + (size_t)idx * 3, a.scale_modifier, a.rotations + (size_t)idx * 4, c6);
    c3 = c6;
  }
  float cv[3];
  cov2d(p, a, c3, cv);
  const float det = cv[0] * cv[2] - cv[1] * cv[1];
  if (det == 0.0f) return 0u;
  const float di = 1.f / det;
  const float mid = 0.5f * (cv[0] + cv[2]);
  const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
  const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
  const int rad = (int)ceilf(3.f * sqrtf(fmaxf(l1, l2)));
  const float px = ndc2pix(ppx, a.W), py = ndc2pix(ppy, a.H);
  int rmin[2], rmax[2];
  get_rect(px, py, rad, a.grid_x, a.grid_y, rmin, rmax);
  if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) return 0u;
  float rgb[3];
  unsigned clamp = 0;
  if (a.colors_precomp) {
    rgb[0] = a.colors_precomp[(size_t)idx * 3 + 0];
    rgb[1] = a.colors_precomp[(size_t)idx * 3 + 1];
    rgb[2] = a.colors_precomp[(size_t)idx * 3 + 2];
  } else {
    if (a.sh_vec4) sh_rgb<true>(a, idx, p, rgb, clamp);
    else sh_rgb<false>(a, idx, p, rgb, clamp);
  }
  depth[idx] = pv[2];
  radii[idx] = rad;
  xy[idx] = make_float2(px, py);
  const float4 co = make_float4(cv[2] * di, -cv[1] * di, cv[0] * di, a.opacities[idx]);
  conic_o[idx] = co;
  rgbo[idx] = make_float4(rgb[0], rgb[1], rgb[2], __uint_as_float(clamp));  // .w: SH clamp bits
  const unsigned full = (unsigned)((rmax[1] - rmin[1]) * (rmax[0] - rmin[0]));
  int t0[2] = {rmin[0], rmin[1]}, t1[2] = {rmax[0], rmax[1]};
  if (a.tight) {
    const Reach rc = reach_of(co);
    if (rc.mode == 1) {
      t1[0] = t0[0];
    } else if (rc.mode == 0) {
      const float lo[2] = {px - rc.ex, py - rc.ey}, hi[2] = {px + rc.ex, py + rc.ey};
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        int first, last;
        reach_cells(lo[d], hi[d], 2 * rmin[d], 2 * rmax[d], first, last);
        t0[d] = first >> 1;
        t1[d] = first > last ? t0[d] : (last >> 1) + 1;
      }
    }
  }
  rect[idx] = pack_rect(t0[0], t0[1], t1[0], t1[1]);
  tiles[idx] = ((unsigned long long)full << 32) | (unsigned)((t1[0] - t0[0]) * (t1[1] - t0[1]));
  return __float_as_uint(pv[2]);
}
// dst (optional): the depth order's min / max shards (dsort.h)
__global__ __launch_bounds__(256) void k_preprocess(RasterDev a, int* __restrict__ radii, float* __restrict__ depth,
                                                    float2* __restrict__ xy, float4* __restrict__ conic_o,
                                                    float4* __restrict__ rgbo, unsigned long long* __restrict__ tiles,
                                                    uint2* __restrict__ rect, unsigned* __restrict__ dst) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned bits = 0u;
  if (idx < a.P) bits = preprocess_one(a, idx, radii, depth, xy, conic_o, rgbo, tiles, rect);
  if (dst) ds_minmax(dst, bits != 0u, bits);  // every lane of the wave: a shuffle reduction
}

__global__ __launch_bounds__(256) void k_duplicate(int P, const uint2* __restrict__ rect, const float* __restrict__ depth,
                                                   const unsigned long long* __restrict__ offsets,
                                                   const int* __restrict__ radii, int gx,
                                                   unsigned long long* __restrict__ keys,
                                                   unsigned* __restrict__ vals) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= P || radii[idx] <= 0) return;
  unsigned off = idx == 0 ? 0u : (unsigned)offsets[idx - 1];
  int rmin[2], rmax[2];
  unpack_rect(rect[idx], rmin, rmax);
  const unsigned dbits = __float_as_uint(depth[idx]);
  for (int y = rmin[1]; y < rmax[1]; ++y)
    for (int x = rmin[0]; x < rmax[0]; ++x) {
      keys[off] = ((unsigned long long)(unsigned)(y * gx + x) << 32) | dbits;
      vals[off] = (unsigned)idx;
      ++off;
    }
}

__global__ __launch_bounds__(256) void k_ranges(int L, const unsigned long long* __restrict__ keys,
                                                uint2* __restrict__ ranges) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= L) return;
  const unsigned cur = (unsigned)(keys[idx] >> 32);
  if (idx == 0) {
    ranges[cur].x = 0;
  } else {
    const unsigned prev = (unsigned)(keys[idx - 1] >> 32);
    if (cur != prev) {
      ranges[prev].y = idx;
      ranges[cur].x = idx;
    }
  }
  if (idx == L - 1) ranges[cur].y = L;
}

// k_render: one wave64 workgroup per 8x8 quarter of a 16x16 tile, walking
// the tile's list front to back in batches of 256 entries, 4 per lane (the
// next batch's gather and the list ids of the one after are in flight while
// a batch blends; with most entries culled a batch blends in less than a
// gather round trip, so batches are sized to cut the round trips).
//
// Sub-tile culling.  A tile's list holds every Gaussian whose 3-sigma rect
// touches the tile, but a faint Gaussian reaches alpha >= 1/255 only inside a
// much smaller ellipse, q = d^T conic d <= 2 ln(255 o).  Each staged entry is
// tested once against the 8x8 sub-tile (the ellipse's bounding box, inflated
// by 2 % and a pixel, so float rounding can never cull a Gaussian the blend
// would take) and the survivors are compacted in list order; the blend walks
// only those.  A culled entry is one upstream's loop skips at every pixel of
// the sub-tile (alpha < 1/255), so pixels, final T and last contributor are
// unchanged.  On the bench's lego frame this removes ~85 % of the per-pixel
// work of the heaviest tiles, whose last contributor sits within the first
// 5-15 % of their list.
//
// Per Gaussian the arithmetic and cut-offs are upstream's; kU Gaussians are
// evaluated independently (their LDS reads and exp2s pipeline) and then folded
// in order, branch-free.
constexpr int kU = 8;
constexpr int kQ = 4;            // list entries per lane per batch
constexpr int kBatch = 64 * kQ;  // entries staged per batch
// k_render's own batch (A/B: GSMPM_RENDER_Q; k_render4 stages kBatch, one entry a lane)
#ifndef GSMPM_RENDER_Q
#define GSMPM_RENDER_Q 4
#endif
constexpr int kQR = GSMPM_RENDER_Q;
constexpr int kBatchR = 64 * kQR;


// Tile keys of the depth-ordered path carry, above the tile index, a mask of
// the tile's four 8x8 sub-tiles the Gaussian can reach (alpha >= 1/255 there,
// reaches_subtile); a pair that reaches none of them gets kCulledKey and is
// sorted out of the tile lists (it is one upstream's blend skips at every
// pixel of the tile).  num_rendered stays upstream's rect count.
constexpr unsigned kMaskShift = 28, kTileField = (1u << kMaskShift) - 1u, kCulledKey = kTileField;
constexpr unsigned kNoEntry = 0xffffffffu;  // id of a chunk-tail slot past K
// Quarter of the workgroup (its 8x8 pixels: column bx, row by in quarters).
// xcd: the four quarters of a tile take linear workgroup ids 32 g + 8 h + x8
// (h: the quarter), so they share id mod 8 -- one XCD (workgroup j runs on
// XCD j mod 8), one L2: the tile's list, its gathered Gaussians and its
// 16-pixel output rows are fetched and merged there once, not in four L2s
// (the row-major grid put a tile's two left/right quarters on two XCDs,
// each writing back half-filled 64-byte lines).  Else the 2-D grid's order.
__device__ __forceinline__ bool render_quarter(int xcd, int gx, int ntiles, int L, int& bx, int& by) {
  if (!xcd) {
    bx = blockIdx.x;
    by = blockIdx.y;
    return true;
  }
  const int x8 = L & 7, h = (L >> 3) & 3, tile = (L >> 5) * 8 + x8;
  if (tile >= ntiles) return false;
  bx = 2 * (tile % gx) + (h & 1);
  by = 2 * (tile / gx) + (h >> 1);
  return true;
}
__global__ __launch_bounds__(64) void k_render(const uint2* __restrict__ ranges, const unsigned* __restrict__ list,
                                               int W, int H, int gx, const float2* __restrict__ xy,
                                               const float4* __restrict__ conic_o, const float4* __restrict__ rgbo,
                                               const float* __restrict__ bg, float* __restrict__ out,
                                               float* __restrict__ final_T, int* __restrict__ n_contrib,
                                               const unsigned* __restrict__ tkeys, int mode, int xcd, int ntiles,
                                               int nq) {
  __shared__ float2 s_xy[kBatchR];
  __shared__ float4 s_co[kBatchR];
  __shared__ float4 s_rgb[kBatchR];  // .w: the entry's tile-list index (as int bits)
  // one quarter per workgroup, or (a grid of fewer workgroups, a multiple of 8
  // so a quarter keeps its XCD) quarters L, L + grid, ...
  for (int L = blockIdx.x; L < nq; L += gridDim.x) {
  int bx, by;
  if (!render_quarter(xcd, gx, ntiles, L, bx, by)) continue;  // workgroup-uniform
  const int lane = threadIdx.x;
  const int x0 = bx * kSub, y0 = by * kSub;
  const int px = x0 + (lane & (kSub - 1)), py = y0 + (lane / kSub);
  const bool inside = px < W && py < H;
  const uint2 range = ranges[(by >> 1) * gx + (bx >> 1)];
  const int n = (int)(range.y - range.x);
  const unsigned* lst = list + range.x;
  const float pfx = (float)px, pfy = (float)py, fx0 = (float)x0, fy0 = (float)y0;
  float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f;
  int last = 0;
  bool done = !inside;
  // lane holds entries j0 + 64 q + lane, q < kQR
  // with tkeys (the depth-ordered sort's keys), an entry's sub-tile mask says
  // whether it reaches this quarter: the gather of one that does not is
  // skipped; without, the quarter test runs on the gathered conic
  const unsigned* tk = tkeys ? tkeys + range.x : nullptr;
  const unsigned qbit = 1u << (kMaskShift + (((by & 1) << 1) | (bx & 1)));
  // The ids and keys of a batch are loaded as raw words and tested only when
  // used, a batch later: testing a key right after its load (a bool kept
  // across the blend) made the compiler wait for each load where it was
  // issued -- the "prefetch" of the next batch's ids and keys stalled the
  // wave for kQR round trips in front of every blend.
  float2 g_xy[kQR];
  float4 g_co[kQR], g_rgb[kQR];
  unsigned gid[kQR], gkey[kQR], nid[kQR], nkey[kQR];
  bool g_rel[kQR];
#pragma unroll
  for (int q = 0; q < kQR; ++q) {  // batch 0's ids and keys, and batch 1's, all issued first
    const bool v0 = 64 * q + lane < n, v1 = kBatchR + 64 * q + lane < n;
    gid[q] = v0 ? lst[64 * q + lane] : 0u;
    gkey[q] = (v0 && tk) ? tk[64 * q + lane] : qbit;
    nid[q] = v1 ? lst[kBatchR + 64 * q + lane] : 0u;
    nkey[q] = (v1 && tk) ? tk[kBatchR + 64 * q + lane] : qbit;
  }
#pragma unroll
  for (int q = 0; q < kQR; ++q) {
    g_xy[q] = make_float2(0.f, 0.f);
    g_co[q] = g_rgb[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    g_rel[q] = 64 * q + lane < n && (gkey[q] & qbit);
    if (g_rel[q]) {
      g_xy[q] = xy[gid[q]];
      g_co[q] = conic_o[gid[q]];
      g_rgb[q] = rgbo[gid[q]];
    }
  }
  for (int j0 = 0; j0 < n; j0 += kBatchR) {
    if (__all(done)) break;
    // stage the batch's survivors in list order; slots up to the next
    // multiple of kU are zero (opacity 0: alpha 0, and fma(0, 0, C) = C)
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < kQR; ++q) {
      const int j = j0 + 64 * q + lane;
      const bool keep = j < n && g_rel[q] && (tk || (mode & 1) || reaches_subtile(g_xy[q], g_co[q], fx0, fy0));
      const unsigned long long m = __ballot(keep);
      const int pos =
          cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (keep) {
        s_xy[pos] = g_xy[q];
        s_co[pos] = g_co[q];
        s_rgb[pos] = make_float4(g_rgb[q].x, g_rgb[q].y, g_rgb[q].z, __int_as_float(j));
      }
      cnt += __popcll(m);
    }
    if (lane < ((cnt + kU - 1) & ~(kU - 1)) - cnt) {
      s_xy[cnt + lane] = make_float2(0.f, 0.f);
      s_co[cnt + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
      s_rgb[cnt + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    // the next batch's gather and the one after's list ids fly while this one blends
    // (every test first -- its words were loaded a batch ago -- then every
    // gather: a test between two gathers is a wait for an older load, which
    // the in-order counter turns into a wait for the gather just issued)
    const float2* pxy[kQR];
    const float4 *pco[kQR], *prgb[kQR];
#pragma unroll
    for (int q = 0; q < kQR; ++q) {
      g_rel[q] = j0 + kBatchR + 64 * q + lane < n && (nkey[q] & qbit);
      pxy[q] = xy + nid[q];
      pco[q] = conic_o + nid[q];
      prgb[q] = rgbo + nid[q];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < kQR; ++q) {
      if (g_rel[q]) {
        g_xy[q] = *pxy[q];
        g_co[q] = *pco[q];
        g_rgb[q] = *prgb[q];
      }
    }
#pragma unroll
    for (int q = 0; q < kQR; ++q) {
      const bool v = j0 + 2 * kBatchR + 64 * q + lane < n;
      nid[q] = v ? lst[j0 + 2 * kBatchR + 64 * q + lane] : 0u;
      nkey[q] = (v && tk) ? tk[j0 + 2 * kBatchR + 64 * q + lane] : qbit;
    }
    for (int b = 0; b < cnt; b += kU) {
      if (__all(done)) break;
      float al[kU];
      float4 c[kU];
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const float2 g = s_xy[b + k];
        const float4 co = s_co[b + k];
        c[k] = s_rgb[b + k];
        const float dx = g.x - pfx, dy = g.y - pfy;
        // the hardware exp2 (v_exp_f32, ~1 ulp): pixel parity is 1e-3, not bitwise
        const float power = __builtin_fmaf(-0.5f, __builtin_fmaf(co.x * dx, dx, co.z * dy * dy), -co.y * dx * dy);
        const float alpha = fminf(0.99f, co.w * __builtin_amdgcn_exp2f(power * 1.4426950408889634f));
        al[k] = (power > 0.0f || alpha < 1.0f / 255.0f) ? 0.f : alpha;
      }
      // front to back, branch-free: a skipped or post-stop Gaussian adds an exact zero
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const float a = done ? 0.f : al[k];
        const float test_T = T * (1 - a);
        const bool stop = a != 0.f && test_T < 0.0001f;
        done = done || stop;
        const bool take = a != 0.f && !stop;
        const float aT = take ? a * T : 0.f;
        C0 = __builtin_fmaf(c[k].x, aT, C0);
        C1 = __builtin_fmaf(c[k].y, aT, C1);
        C2 = __builtin_fmaf(c[k].z, aT, C2);
        T = take ? test_T : T;
        last = take ? __float_as_int(c[k].w) + 1 : last;
      }
    }
    __syncthreads();
  }
  if (inside) {
    const size_t pix = (size_t)py * W + px, HW = (size_t)H * W;
    out[pix] = C0 + T * bg[0];
    out[HW + pix] = C1 + T * bg[1];
    out[2 * HW + pix] = C2 + T * bg[2];
    if (final_T) {  // the backward's per-pixel state; a forward-only context skips it
      final_T[pix] = T;
      n_contrib[pix] = last;
    }
  }
  }
}

// k_render4: the same blend, one 256-lane workgroup per tile, wave q = the
// tile's 8x8 quarter q.  Each batch of kBatch list entries is read ONCE per
// tile: lane t loads entry j0 + t's id and sub-tile mask and, if any quarter
// wants it, gathers its xy / conic / rgb into LDS (k_render's four quarter
// workgroups each read the whole list and gather their own reachers, up to
// 4x the bytes).  Each wave then compacts its quarter's survivors, in list
// order, as indices into the staged batch and blends them exactly as
// k_render does (same arithmetic, same order: bit-identical pixels, final T
// and last contributor).  Staging is double-buffered: one barrier a batch,
// and the next batch's gathers are in flight while this one blends.  The
// workgroup stops when all 256 pixels are done.
constexpr int kStage = kBatch + kU;  // + kU all-zero slots: the padding of a wave's last group of kU
__global__ __launch_bounds__(256) void k_render4(const uint2* __restrict__ ranges, const unsigned* __restrict__ list,
                                                 int W, int H, int gx, const float2* __restrict__ xy,
                                                 const float4* __restrict__ conic_o, const float4* __restrict__ rgbo,
                                                 const float* __restrict__ bg, float* __restrict__ out,
                                                 float* __restrict__ final_T, int* __restrict__ n_contrib,
                                                 const unsigned* __restrict__ tkeys, int mode) {
  __shared__ float2 s_xy[2][kStage];
  __shared__ float4 s_co[2][kStage];
  __shared__ float4 s_rgb[2][kStage];  // .w: the entry's tile-list index (as int bits)
  __shared__ unsigned char s_m[2][kBatch];
  __shared__ unsigned short s_idx[4][kBatch + kU];
  const int t = threadIdx.x, lane = t & 63, q = t >> 6;
  const int x0 = blockIdx.x * kBX + (q & 1) * kSub, y0 = blockIdx.y * kBY + (q >> 1) * kSub;
  const int px = x0 + (lane & (kSub - 1)), py = y0 + (lane / kSub);
  const bool inside = px < W && py < H;
  const uint2 range = ranges[blockIdx.y * gx + blockIdx.x];
  const int n = (int)(range.y - range.x);
  const unsigned* lst = list + range.x;
  const unsigned* tk = tkeys ? tkeys + range.x : nullptr;
  const float pfx = (float)px, pfy = (float)py, fx0 = (float)x0, fy0 = (float)y0;
  float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f;
  int last = 0;
  bool done = !inside;
  if (t < kU)
    for (int b = 0; b < 2; ++b) {
      s_xy[b][kBatch + t] = make_float2(0.f, 0.f);
      s_co[b][kBatch + t] = make_float4(0.f, 0.f, 0.f, 0.f);
      s_rgb[b][kBatch + t] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  // lane t's entry of the current batch (gathered) and of the next (id, mask)
  float2 g_xy = make_float2(0.f, 0.f);
  float4 g_co = make_float4(0.f, 0.f, 0.f, 0.f), g_rgb = g_co;
  unsigned g_m = 0, n_id = 0, n_m = 0;
  auto mask_of = [&](int j) -> unsigned { return tk ? (tk[j] >> kMaskShift) & 0xfu : 0xfu; };
  if (t < n) {
    g_m = mask_of(t);
    if (g_m) {
      const unsigned id = lst[t];
      g_xy = xy[id];
      g_co = conic_o[id];
      g_rgb = rgbo[id];
    }
  }
  if (kBatch + t < n) {
    n_id = lst[kBatch + t];
    n_m = mask_of(kBatch + t);
  }
  int buf = 0;
  for (int j0 = 0; j0 < n; j0 += kBatch, buf ^= 1) {
    s_xy[buf][t] = g_xy;
    s_co[buf][t] = g_co;
    s_rgb[buf][t] = make_float4(g_rgb.x, g_rgb.y, g_rgb.z, __int_as_float(j0 + t));
    s_m[buf][t] = (unsigned char)(j0 + t < n ? g_m : 0u);
    if (__syncthreads_count(!done) == 0) break;
    // the next batch's gather and the one after's ids fly while this one blends
    g_m = j0 + kBatch + t < n ? n_m : 0u;
    if (g_m) {
      g_xy = xy[n_id];
      g_co = conic_o[n_id];
      g_rgb = rgbo[n_id];
    }
    if (j0 + 2 * kBatch + t < n) {
      n_id = lst[j0 + 2 * kBatch + t];
      n_m = mask_of(j0 + 2 * kBatch + t);
    }
    // this quarter's survivors of the staged batch, in list order
    int cnt = 0;
#pragma unroll
    for (int r = 0; r < kBatch / 64; ++r) {
      const int e = r * 64 + lane;
      bool keep = (s_m[buf][e] >> q) & 1u;
      if (keep && !tk && !(mode & 1)) keep = reaches_subtile(s_xy[buf][e], s_co[buf][e], fx0, fy0);
      const unsigned long long m = __ballot(keep);
      const int pos =
          cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (keep) s_idx[q][pos] = (unsigned short)e;
      cnt += __popcll(m);
    }
    if (lane < ((cnt + kU - 1) & ~(kU - 1)) - cnt) s_idx[q][cnt + lane] = (unsigned short)(kBatch + lane);
#ifdef GSMPM_RENDER4_BARRIER
    __syncthreads();
#else
    // s_idx is this wave's own: its LDS writes complete (in order) before its reads
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    for (int b = 0; b < cnt; b += kU) {
      if (__all(done)) break;
      float al[kU];
      float4 c[kU];
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const int e = s_idx[q][b + k];
        const float2 g = s_xy[buf][e];
        const float4 co = s_co[buf][e];
        c[k] = s_rgb[buf][e];
        const float dx = g.x - pfx, dy = g.y - pfy;
        const float power = __builtin_fmaf(-0.5f, __builtin_fmaf(co.x * dx, dx, co.z * dy * dy), -co.y * dx * dy);
        const float alpha = fminf(0.99f, co.w * __builtin_amdgcn_exp2f(power * 1.4426950408889634f));
        al[k] = (power > 0.0f || alpha < 1.0f / 255.0f) ? 0.f : alpha;
      }
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const float a = done ? 0.f : al[k];
        const float test_T = T * (1 - a);
        const bool stop = a != 0.f && test_T < 0.0001f;
        done = done || stop;
        const bool take = a != 0.f && !stop;
        const float aT = take ? a * T : 0.f;
        C0 = __builtin_fmaf(c[k].x, aT, C0);
        C1 = __builtin_fmaf(c[k].y, aT, C1);
        C2 = __builtin_fmaf(c[k].z, aT, C2);
        T = take ? test_T : T;
        last = take ? __float_as_int(c[k].w) + 1 : last;
      }
    }
  }
  if (inside) {
    const size_t pix = (size_t)py * W + px, HW = (size_t)H * W;
    out[pix] = C0 + T * bg[0];
    out[HW + pix] = C1 + T * bg[1];
    out[2 * HW + pix] = C2 + T * bg[2];
    if (final_T) {
      final_T[pix] = T;
      n_contrib[pix] = last;
    }
  }
}

constexpr unsigned kNoCount = 0xffffffffu;
// dst[1] = the 3-sigma pair count (num_rendered), dst[2] = the depth order's
// overflow flag (dsort.h; null: 0), then dst[0] = the binned count K (the host spins on it)
__global__ void k_publish_count(const unsigned long long* __restrict__ src, const unsigned* __restrict__ over,
                                unsigned* dst) {
  const unsigned long long v = *src;
  __hip_atomic_store(dst + 2, over ? *over : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(dst + 1, (unsigned)(v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(dst, (unsigned)v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the async form with no Gaussians: the background, and every count 0
__global__ __launch_bounds__(256) void k_fill_bg(const float* __restrict__ bg, int npix, float* __restrict__ out,
                                                 unsigned* counts) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < npix) {
    out[i] = bg[0];
    out[npix + i] = bg[1];
    out[2 * npix + i] = bg[2];
  }
  if (i < 4) counts[i] = 0u;
}

// sorted emission index -> Gaussian id (the sort carries emission indices)
__global__ __launch_bounds__(256) void k_ids(int K, const unsigned* __restrict__ pos, const unsigned* __restrict__ vals,
                                             unsigned* __restrict__ ids) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < K) ids[k] = vals[pos[k]];
}

// Depth-ordered emission (the default binning path).  The Gaussians are
// first sorted by depth (stable, so equal depths keep index order); each then
// emits its rect's pairs at its offset in that order, and a stable sort on the
// tile index alone (msb(#tiles) bits, two onesweep passes) leaves every tile's
// list in (depth, Gaussian index) order -- the list upstream's 64-bit
// (tile << 32 | depth bits) sort produces, with 4-byte keys and 12 bits of
// radix instead of 32 + 12.
// tiles touched by the Gaussian of depth rank r: the depth-order scan's input
// (both counts of k_preprocess's tiles word: their scan's last entry holds K and num_rendered)
struct TilesOfRank {
  const unsigned long long* tiles;
  __host__ __device__ unsigned long long operator()(unsigned g) const { return tiles[g]; }
};
inline rocprim::transform_iterator<const unsigned*, TilesOfRank, unsigned long long> ranked_tiles(
    const unsigned* order, const unsigned long long* tiles) {
  return rocprim::transform_iterator<const unsigned*, TilesOfRank, unsigned long long>(order, TilesOfRank{tiles});
}
// the binned count alone (the index-order offsets of the record slots)
struct BinnedTiles {
  __host__ __device__ unsigned operator()(unsigned long long t) const { return (unsigned)t; }
};
inline rocprim::transform_iterator<const unsigned long long*, BinnedTiles, unsigned> binned_tiles(
    const unsigned long long* tiles) {
  return rocprim::transform_iterator<const unsigned long long*, BinnedTiles, unsigned>(tiles, BinnedTiles{});
}
// Depth-ordered emission, one lane per pair (a lane per Gaussian would
// serialise the ~1600 stores of the frame's largest Gaussians): the pair's
// Gaussian is found by binary search over the depth-order offsets, and the
// pair lands at its depth-order offset + its index in the Gaussian's rect.
__global__ __launch_bounds__(256) void k_emit_pairs(int K, int P, const unsigned* __restrict__ order,
                                                    const unsigned long long* __restrict__ offr,
                                                    const float2* __restrict__ xy, const float4* __restrict__ conic_o,
                                                    const uint2* __restrict__ rect, int gx, int cull,
                                                    unsigned* __restrict__ keys, unsigned* __restrict__ ids) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= K) return;
  int lo = 0, hi = P - 1;  // first r with offr[r] > e (offr: inclusive scan)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((unsigned)offr[mid] > (unsigned)e) hi = mid;
    else lo = mid + 1;
  }
  const unsigned g = order ? order[lo] : (unsigned)lo;
  const unsigned local = (unsigned)e - (lo ? (unsigned)offr[lo - 1] : 0u);
  const float2 gp = xy[g];
  int rmin[2], rmax[2];
  unpack_rect(rect[g], rmin, rmax);
  const unsigned w = (unsigned)(rmax[0] - rmin[0]);
  const int x = rmin[0] + (int)(local % w), y = rmin[1] + (int)(local / w);
  unsigned m = 0xfu;
  if (cull) {
    const Reach rc = reach_of(conic_o[g]);
    m = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (reaches_box(rc, gp, (float)(x * kBX + (q & 1) * kSub), (float)(y * kBY + (q >> 1) * kSub))) m |= 1u << q;
  }
  keys[e] = m ? ((unsigned)(y * gx + x) | (m << kMaskShift)) : kCulledKey;
  ids[e] = g;
}
// Balanced depth-ordered emission (the default; k_emit_pairs above stays for
// GSMPM_RASTER_EMIT_LANE=1).  k_emit_pairs' per-lane binary search is a
// ~20-deep chain of dependent global loads at 1M Gaussians: bicycle's 39M
// pairs took 546 us, memory-wait bound (SQ_WAIT_ANY 75 %).  Here a workgroup
// owns `items` x 256 consecutive pairs [e0, e1):
//   - the Gaussians r0 / r1 of its first and last pair come from
//     k_emit_starts (the Gaussian holding each workgroup's first pair,
//     written by that Gaussian's lane; a cooperative 256-ary search per
//     workgroup cost six dependent round trips before any work started);
//   - the Gaussians [r0, r1] are staged in LDS, kEmitG at a time: offsets,
//     id, tile rect and (culling) the alpha-reach box, one coalesced round
//     of loads per Gaussian instead of one per pair;
//   - each pair of the staged span finds its Gaussian by a binary search in
//     LDS (from the lane's previous one) and is emitted from LDS alone.
// Same pairs, same positions, same keys as k_emit_pairs.
#ifndef GSMPM_EMIT_G
#define GSMPM_EMIT_G 512  // 16 KB of staging: 8 workgroups per CU (1024: 4 per CU, bicycle k_emit_wg 133 vs 114 us)
#endif
constexpr int kEmitT = 256, kEmitMaxI = 16, kEmitG = GSMPM_EMIT_G;
// starts[b] = the depth rank of the Gaussian holding pair b * E (E = pairs per
// emission workgroup): each boundary lies in exactly one non-empty Gaussian
// The async form (gsmpm_raster_forward_async: the pair count stays on the
// device): at most bmax starts are written, and the lane of the last Gaussian
// raises bit 1 of *flags when the frame bins more pairs than kcap (the pair
// buffers were carved for kcap: the emission and the tile sort cut at kcap and
// the caller renders the frame again with room for the count).
__global__ __launch_bounds__(256) void k_emit_starts(int P, const unsigned long long* __restrict__ offr, unsigned E,
                                                     unsigned* __restrict__ starts, unsigned bmax, unsigned kcap,
                                                     const unsigned* __restrict__ over, unsigned* flags) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= P) return;
  const unsigned s = r ? (unsigned)offr[r - 1] : 0u, t = (unsigned)offr[r];
  for (unsigned b = (s + E - 1) / E; b * E < t && b < bmax; ++b) starts[b] = (unsigned)r;
  // the whole flags word, one store (the depth order's bucket overflow from the
  // device state, not read back from the caller's host memory)
  if (flags && r == P - 1) flags[0] = (over ? *over : 0u) | (t > kcap ? 2u : 0u);
}
// K of the frame: the host's count, or (the async form) the device's, cut at the host's capacity
__device__ __forceinline__ int pairs_of(int K, const unsigned long long* kdev) {
  return kdev ? min(K, (int)min((unsigned)*kdev, 0x7fffffffu)) : K;
}
__global__ __launch_bounds__(kEmitT) void k_emit_wg(int K, int P, int items, const unsigned* __restrict__ starts,
                                                    const unsigned* __restrict__ order,
                                                    const unsigned long long* __restrict__ offr,
                                                    const float2* __restrict__ xy, const float4* __restrict__ conic_o,
                                                    const uint2* __restrict__ rect, int gx, int cull,
                                                    unsigned* __restrict__ keys, unsigned* __restrict__ ids,
                                                    const unsigned long long* __restrict__ kdev) {
  __shared__ unsigned s_off[kEmitG + 1];  // [i]: first pair of staged Gaussian i, [i + 1]: one past its last
  __shared__ unsigned s_g[kEmitG];        // Gaussian id
  __shared__ uint2 s_rect[kEmitG];        // (x0 | y0 << 16, rect width) in tiles
  __shared__ float4 s_box[kEmitG];        // alpha-reach box (x lo, x hi, y lo, y hi) in pixels (culling)
  K = pairs_of(K, kdev);
  const int e0 = blockIdx.x * kEmitT * items, e1 = min(K, e0 + kEmitT * items);
  if (e0 >= K) return;  // the async form's workgroups past the frame's pairs (uniform)
  const int r0 = (int)starts[blockIdx.x];
  const int r1 = e1 < K ? (int)starts[blockIdx.x + 1] : P - 1;  // may stage one Gaussian past pair e1 - 1
  int rs = r0;        // first Gaussian of the span to stage
  unsigned pa = e0;   // first pair not yet emitted
  while (true) {      // uniform: spans of <= kEmitG Gaussians
    const int ns = min(kEmitG, r1 + 1 - rs);
    __syncthreads();  // the previous span's readers are done
    if (threadIdx.x == 0) s_off[0] = rs ? (unsigned)offr[rs - 1] : 0u;
    for (int i = threadIdx.x; i < ns; i += kEmitT) {
      const unsigned g = order ? order[rs + i] : (unsigned)(rs + i);  // null: Gaussian-index order
      s_off[i + 1] = (unsigned)offr[rs + i];
      s_g[i] = g;
      const uint2 rr = rect[g];
      s_rect[i] = make_uint2(rr.x, (unsigned)max((int)(rr.y & 0xffffu) - (int)(rr.x & 0xffffu), 1));
      if (cull) {
        const float2 gp = xy[g];  // reaches_box's comparisons on the same sums (mode 1: empty box, mode 2: everything)
        const Reach rc = reach_of(conic_o[g]);
        const float inf = __builtin_inff();
        s_box[i] = rc.mode == 1   ? make_float4(inf, -inf, inf, -inf)
                   : rc.mode == 2 ? make_float4(-inf, inf, -inf, inf)
                                  : make_float4(gp.x - rc.ex, gp.x + rc.ex, gp.y - rc.ey, gp.y + rc.ey);
      }
    }
    __syncthreads();
    const unsigned pb = min((unsigned)e1, s_off[ns]);
    int lo = 0;
    for (unsigned e = pa + threadIdx.x; e < pb; e += kEmitT) {
      int hi = ns - 1;  // first i with s_off[i + 1] > e (exists: e < s_off[ns])
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_off[mid + 1] > e) hi = mid;
        else lo = mid + 1;
      }
      const uint2 rw = s_rect[lo];
      const unsigned local = e - s_off[lo];
      const int x = (int)(rw.x & 0xffffu) + (int)(local % rw.y), y = (int)(rw.x >> 16) + (int)(local / rw.y);
      unsigned m = 0xfu;
      if (cull) {
        const float4 bx = s_box[lo];
        m = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float x0 = (float)(x * kBX + (q & 1) * kSub), y0 = (float)(y * kBY + (q >> 1) * kSub);
          if (!(bx.y < x0 || bx.x > x0 + (kSub - 1) || bx.w < y0 || bx.z > y0 + (kSub - 1))) m |= 1u << q;
        }
      }
      keys[e] = m ? ((unsigned)(y * gx + x) | (m << kMaskShift)) : kCulledKey;
      ids[e] = s_g[lo];
    }
    pa = pb;
    rs += ns;
    if (pa >= (unsigned)e1) break;
  }
}
// Stable tile sort of the depth-ordered emission list for <= kMaxTiles tiles
// (replaces the two onesweep passes: 2 kernels + a scan instead of ~8
// launches, no look-back chain).  The list is cut into chunks of kChunk pairs.
//   k_tile_hist     per chunk, the pair count of every tile (LDS atomics),
//                   stored tile-major: H[t * nch + c]
//   exclusive scan  over H -> the output position of chunk c's first pair of
//                   tile t (tile-major order = sorted order)
//   k_tile_scatter  per chunk, a stable block radix sort on the tile bits in
//                   LDS; a pair at sorted position s of run [s0, ..) of tile t
//                   lands at H'[t * nch + c] + s - s0.  Chunk 0 also writes
//                   every tile's [start, end).
constexpr int kMaxTiles = 4096, kSortT = 256, kSortI = 8, kChunk = kSortT * kSortI;
// culled pairs count as a virtual tile `ntiles` (sorted after every real
// tile, so [0, K) of the output stays fully written)
__device__ __forceinline__ unsigned sort_tile(unsigned key, unsigned lowmask, int ntiles) {
  const unsigned t = key & lowmask;
  return t < (unsigned)ntiles ? t : (unsigned)ntiles;
}
// a block sort's blocked result (thread t holds sorted positions t * kSortI + i)
// to LDS in sorted order: two 16-byte stores of keys and of values per thread
__device__ __forceinline__ void sorted_to_lds(const unsigned (&k)[kSortI], const unsigned (&v)[kSortI],
                                              unsigned* s_k, unsigned* s_v) {
  static_assert(kSortI == 8, "two uint4 per thread");
  uint4* dk = reinterpret_cast<uint4*>(s_k + threadIdx.x * kSortI);
  uint4* dv = reinterpret_cast<uint4*>(s_v + threadIdx.x * kSortI);
  dk[0] = make_uint4(k[0], k[1], k[2], k[3]);
  dk[1] = make_uint4(k[4], k[5], k[6], k[7]);
  dv[0] = make_uint4(v[0], v[1], v[2], v[3]);
  dv[1] = make_uint4(v[4], v[5], v[6], v[7]);
  __syncthreads();
}
__global__ __launch_bounds__(kSortT) void k_tile_hist(int K, int ntiles, int nch, int bits,
                                                      const unsigned* __restrict__ keys, unsigned* __restrict__ H,
                                                      const unsigned long long* __restrict__ kdev) {
  __shared__ unsigned s_h[kMaxTiles + 1];
  K = pairs_of(K, kdev);  // chunks past the frame's pairs store empty histograms
  const unsigned lowmask = (1u << bits) - 1u;
  for (int t = threadIdx.x; t <= ntiles; t += kSortT) s_h[t] = 0;
  __syncthreads();
  const int c = blockIdx.x;
  // every key of the chunk loaded first (clamped indices), then the counts:
  // a load then its atomic per element made the compiler wait on each load,
  // kChunk / kSortT round trips in a row
  constexpr int kPer = kChunk / kSortT;
  unsigned kv[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) kv[u] = keys[min(c * kChunk + (int)threadIdx.x + u * kSortT, max(K - 1, 0))];
#pragma unroll
  for (int u = 0; u < kPer; ++u)
    if (c * kChunk + (int)threadIdx.x + u * kSortT < K) atomicAdd(&s_h[sort_tile(kv[u], lowmask, ntiles)], 1u);
  __syncthreads();
  for (int t = threadIdx.x; t <= ntiles; t += kSortT) H[(size_t)t * nch + c] = s_h[t];
}
// GSMPM_TILE_BRS=1 (A/B build): the chunk's stable order from the library's
// block radix sort instead of the wave-ballot ranks below
#ifndef GSMPM_TILE_BRS
#define GSMPM_TILE_BRS 0
#endif
__global__ __launch_bounds__(kSortT) void k_tile_scatter(int K, int ntiles, int nch, int bits,
                                                         const unsigned* __restrict__ keys,
                                                         const unsigned* __restrict__ vals,
                                                         const unsigned* __restrict__ Hs,
                                                         const unsigned* __restrict__ tot,
                                                         unsigned* __restrict__ keys_out, unsigned* __restrict__ vals_out,
                                                         uint2* __restrict__ ranges, int* __restrict__ dsort_counts,
                                                         const unsigned long long* __restrict__ kdev) {
  if (dsort_counts && blockIdx.x == 0 && threadIdx.x < 2) dsort_counts[threadIdx.x] = 0;  // k_tile_dsort's lists
  K = pairs_of(K, kdev);
  __shared__ unsigned s_k[kChunk], s_v[kChunk];
  __shared__ int s_start[kMaxTiles + 1];    // chunk-local start of each tile's run
  __shared__ unsigned s_ts[kMaxTiles + 2];  // exclusive scan of the tile totals: each tile's run start
  __shared__ unsigned s_part[kSortT];
  const int c = blockIdx.x;
  const unsigned lowmask = (1u << bits) - 1u;  // >= ntiles
  {
    // the thread's <= 17 tile totals loaded at once (clamped indices), kept in
    // registers for the second pass: loaded in a loop with the sum, each load
    // was waited for before the next
    constexpr int kPerMax = (kMaxTiles + 1 + kSortT - 1) / kSortT;
    const int per = (ntiles + 1 + kSortT - 1) / kSortT, t0 = threadIdx.x * per;
    unsigned tv[kPerMax];
#pragma unroll
    for (int q = 0; q < kPerMax; ++q) tv[q] = tot[min(t0 + q, ntiles)];
    unsigned sum = 0;
#pragma unroll
    for (int q = 0; q < kPerMax; ++q) sum += (q < per && t0 + q <= ntiles) ? tv[q] : 0u;
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < kSortT; o <<= 1) {
      const unsigned u = threadIdx.x >= (unsigned)o ? s_part[threadIdx.x - o] : 0u;
      __syncthreads();
      s_part[threadIdx.x] += u;
      __syncthreads();
    }
    unsigned run = s_part[threadIdx.x] - sum;
#pragma unroll
    for (int q = 0; q < kPerMax; ++q)
      if (q < per && t0 + q <= ntiles) {
        s_ts[t0 + q] = run;
        run += tv[q];
      }
    if (threadIdx.x == kSortT - 1) s_ts[ntiles + 1] = run;
  }
#if GSMPM_TILE_BRS
  using BRS = rocprim::block_radix_sort<unsigned, kSortT, kSortI, unsigned>;
  __shared__ typename BRS::storage_type s_sort;
  unsigned k[kSortI], v[kSortI];
#pragma unroll
  for (int i = 0; i < kSortI; ++i) {
    const int e = c * kChunk + threadIdx.x * kSortI + i;  // blocked: the sort is stable in this order
    k[i] = e < K ? keys[e] : kNoEntry;
    v[i] = e < K ? vals[e] : kNoEntry;
  }
  BRS().sort(k, v, s_sort, 0, bits);
  sorted_to_lds(k, v, s_k, s_v);
  // sorted position sp is read striped (sp = i * kSortT + lane): a run's pairs
  // go out as coalesced stores (the blocked order wrote 64 lanes 32 B apart)
#pragma unroll
  for (int i = 0; i < kSortI; ++i) {
    const int sp = i * kSortT + threadIdx.x;
    const unsigned t = sort_tile(s_k[sp], lowmask, ntiles);
    if (s_v[sp] != kNoEntry && (sp == 0 || sort_tile(s_k[sp - 1], lowmask, ntiles) != t)) s_start[t] = sp;
  }
  __syncthreads();
#else
  // The chunk's stable order by tile, without a block sort: wave w ranks its
  // 512 pairs [w * 512, +512) of the chunk in 8 slots of 64, in order, by
  // matching lanes of equal tile with 13 ballots and a wave-private running
  // count per tile (LDS); the four waves' counts then give every tile's run
  // start in the chunk and each wave's offset inside it.  The rank follows
  // (wave, slot, lane) = the chunk's order: stable, as the block sort was.
  __shared__ unsigned s_cnt[4][kMaxTiles + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < 4 * (kMaxTiles + 1); e += kSortT) (&s_cnt[0][0])[e] = 0u;
  __syncthreads();
  constexpr int kW = kChunk / 4;  // pairs per wave
  const int e0 = c * kChunk + wv * kW;
  unsigned k[kSortI], v[kSortI], r[kSortI], tl[kSortI];
#pragma unroll
  for (int j = 0; j < kSortI; ++j) {  // unconditional loads (clamped), then the selects: no wait between them
    const int ec = min(e0 + j * 64 + lane, max(K - 1, 0));
    k[j] = keys[ec];
    v[j] = vals[ec];
  }
#pragma unroll
  for (int j = 0; j < kSortI; ++j) {
    const int e = e0 + j * 64 + lane;
    k[j] = e < K ? k[j] : 0u;
    v[j] = e < K ? v[j] : 0u;
    tl[j] = e < K ? sort_tile(k[j], lowmask, ntiles) : 8191u;  // 8191: no pair (13 bits, > any tile)
  }
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < kSortI; ++j) {
    const unsigned d = tl[j];
    unsigned long long peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 13; ++b) {
      const unsigned long long bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const unsigned rk = (unsigned)__popcll(peers & below);
    const bool ok = d != 8191u;
    const unsigned base = ok ? s_cnt[wv][d] : 0u;
    r[j] = base + rk;
    // the tile's lowest lane moves the count on (the wave's LDS operations are in order)
    if (ok && rk == 0) s_cnt[wv][d] = base + (unsigned)__popcll(peers);
  }
  __syncthreads();
  {  // per tile: the run start in the chunk (scan of the four waves' counts) and each wave's offset
    const int per = (ntiles + 1 + kSortT - 1) / kSortT, t0 = threadIdx.x * per;
    unsigned sum = 0;
    for (int q = 0; q < per; ++q)
      if (t0 + q <= ntiles) sum += s_cnt[0][t0 + q] + s_cnt[1][t0 + q] + s_cnt[2][t0 + q] + s_cnt[3][t0 + q];
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < kSortT; o <<= 1) {
      const unsigned u = threadIdx.x >= (unsigned)o ? s_part[threadIdx.x - o] : 0u;
      __syncthreads();
      s_part[threadIdx.x] += u;
      __syncthreads();
    }
    unsigned run = s_part[threadIdx.x] - sum;
    for (int q = 0; q < per; ++q)
      if (t0 + q <= ntiles) {
        const int t = t0 + q;
        const unsigned c0 = s_cnt[0][t], c1 = s_cnt[1][t], c2 = s_cnt[2][t], c3 = s_cnt[3][t];
        s_start[t] = (int)run;
        s_cnt[0][t] = run;
        s_cnt[1][t] = run + c0;
        s_cnt[2][t] = run + c0 + c1;
        s_cnt[3][t] = run + c0 + c1 + c2;
        run += c0 + c1 + c2 + c3;
      }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSortI; ++j)
    if (tl[j] != 8191u) {
      const unsigned idx = s_cnt[wv][tl[j]] + r[j];
      s_k[idx] = k[j];
      s_v[idx] = v[j];
    }
  const int nv = max(0, min(kChunk, K - c * kChunk));  // 0: an async-form chunk past the frame's pairs
  for (int sp = nv + (int)threadIdx.x; sp < kChunk; sp += kSortT) s_v[sp] = kNoEntry;  // the tail: no pair
  __syncthreads();
#endif
  // every chunk-offset load first (a no-pair slot reads tile 0's), then the
  // stores: a load, its wait and its store per slot were kSortI round trips
  unsigned hv[kSortI], tv[kSortI];
#pragma unroll
  for (int i = 0; i < kSortI; ++i) {
    const int sp = i * kSortT + threadIdx.x;
    const unsigned t = s_v[sp] == kNoEntry ? 0u : sort_tile(s_k[sp], lowmask, ntiles);
    tv[i] = t;
    hv[i] = Hs[(size_t)t * nch + c];
  }
#pragma unroll
  for (int i = 0; i < kSortI; ++i) {
    const int sp = i * kSortT + threadIdx.x;
    const unsigned vv = s_v[sp];
    if (vv == kNoEntry) continue;
    const unsigned t = tv[i];
    const unsigned pos = s_ts[t] + hv[i] + (unsigned)(sp - s_start[t]);
    keys_out[pos] = s_k[sp];
    vals_out[pos] = vv;
  }
  if (c == 0)
    for (int tt = threadIdx.x; tt < ntiles; tt += kSortT) ranges[tt] = make_uint2(s_ts[tt], s_ts[tt + 1]);
}

// Per-tile depth order (chunked path, opt-in with GSMPM_RASTER_TILE_DSORT=1; off by
// default: bit-identical but slower, lego render 0.311 vs 0.194 ms).
// Pairs are emitted in Gaussian-index order and the stable tile sort keeps it,
// so each tile's list comes out in index order; sorting each list by the
// composite (depth bits << 32 | position) -- unique, and position order is
// index order -- gives exactly the (depth, index) order a global stable depth
// sort of the Gaussians followed by emission in that order produced, without
// the global sort (rocPRIM's block sort + merge passes over all P depths).
// Lists of <= CAP entries are sorted in LDS by a bitonic network (tiles with
// (lo, CAP] entries: two launches, a small and a large LDS class); longer ones
// by k_tile_dsort_rank.  Depths are > 0.2 (k_preprocess culls nearer ones), so
// their bits order as the floats do.
// tl: [0] tiles listed for the large class, [1] for k_tile_dsort_rank, then
// the two lists of ntiles entries each (k_tile_scatter's chunk 0 zeroes the
// counts).  The small class walks every tile and lists the longer ones; the
// large class walks its list and lists the longer ones for the rank kernel.
template <int CAP, bool LISTED>
__global__ __launch_bounds__(256) void k_tile_dsort(const uint2* __restrict__ ranges, int ntiles,
                                                    const float* __restrict__ depth, unsigned* __restrict__ keys,
                                                    unsigned* __restrict__ ids, int* __restrict__ tl) {
  __shared__ unsigned long long s_c[CAP];
  __shared__ unsigned s_id[CAP], s_key[CAP];
  const int nt = LISTED ? tl[0] : ntiles;
  for (int w = blockIdx.x; w < nt; w += gridDim.x) {
    const int t = LISTED ? tl[2 + w] : w;
    const uint2 rg = ranges[t];
    const int n = (int)(rg.y - rg.x);
    if (n > CAP) {  // workgroup-uniform: the next class
      if (threadIdx.x == 0) {
        const int i = atomicAdd(&tl[LISTED ? 1 : 0], 1);
        tl[2 + (LISTED ? ntiles : 0) + i] = t;
      }
      continue;
    }
    if (n <= 1) continue;
    int m = 2;
    while (m < n) m <<= 1;
    __syncthreads();  // the previous tile's readers are done
    for (int j = threadIdx.x; j < m; j += 256) {
      if (j < n) {
        const unsigned id = ids[rg.x + j];
        s_id[j] = id;
        s_key[j] = keys[rg.x + j];
        s_c[j] = ((unsigned long long)__float_as_uint(depth[id]) << 32) | (unsigned)j;
      } else {
        s_c[j] = ~0ull;
      }
    }
    __syncthreads();
    for (int k = 2; k <= m; k <<= 1)
      for (int h = k >> 1; h > 0; h >>= 1) {
        for (int i = threadIdx.x; i < m; i += 256) {
          const int ix = i ^ h;
          if (ix > i) {
            const unsigned long long a = s_c[i], b = s_c[ix];
            if ((a > b) == ((i & k) == 0)) {
              s_c[i] = b;
              s_c[ix] = a;
            }
          }
        }
        __syncthreads();
      }
    for (int j = threadIdx.x; j < n; j += 256) {
      const unsigned p = (unsigned)s_c[j];
      ids[rg.x + j] = s_id[p];
      keys[rg.x + j] = s_key[p];
    }
  }
}
// Lists longer than the large LDS class (rare): each entry's rank among its
// tile's composites, counted against the whole list (O(n^2) per tile), into
// scratch, then copied back.
constexpr int kDsortSmall = 1024, kDsortLarge = 8192;
__global__ __launch_bounds__(256) void k_tile_dsort_rank(const uint2* __restrict__ ranges, int ntiles,
                                                         const float* __restrict__ depth,
                                                         unsigned* __restrict__ keys, unsigned* __restrict__ ids,
                                                         const int* __restrict__ tl, unsigned* __restrict__ scr_keys,
                                                         unsigned* __restrict__ scr_ids) {
  for (int w = blockIdx.x; w < tl[1]; w += gridDim.x) {
    const int t = tl[2 + ntiles + w];
    const uint2 rg = ranges[t];
    const int n = (int)(rg.y - rg.x);
    for (int j = threadIdx.x; j < n; j += 256) {
      const unsigned long long cj = ((unsigned long long)__float_as_uint(depth[ids[rg.x + j]]) << 32) | (unsigned)j;
      int r = 0;
      for (int i = 0; i < n; ++i)
        r += (((unsigned long long)__float_as_uint(depth[ids[rg.x + i]]) << 32) | (unsigned)i) < cj;
      scr_ids[rg.x + r] = ids[rg.x + j];
      scr_keys[rg.x + r] = keys[rg.x + j];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += 256) {
      ids[rg.x + j] = scr_ids[rg.x + j];
      keys[rg.x + j] = scr_keys[rg.x + j];
    }
    __syncthreads();
  }
}

// backward only: sorted pair -> its record slot, the pair's index in
// Gaussian-index emission order (k_preprocess_bwd sums each Gaussian's
// contiguous slots without atomics)
__global__ __launch_bounds__(256) void k_slots(int K, const unsigned* __restrict__ tile_sorted,
                                               const unsigned* __restrict__ ids, const uint2* __restrict__ rect,
                                               const unsigned* __restrict__ offsets, int gx, int gy,
                                               unsigned* __restrict__ pos) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const unsigned id = ids[k], tile = tile_sorted[k] & kTileField;
  if (tile >= (unsigned)(gx * gy)) return;  // a culled pair (in no tile list)
  int rmin[2], rmax[2];
  unpack_rect(rect[id], rmin, rmax);
  const int tx = (int)(tile % (unsigned)gx), ty = (int)(tile / (unsigned)gx);
  pos[k] = (id == 0 ? 0u : offsets[id - 1]) + (unsigned)((ty - rmin[1]) * (rmax[0] - rmin[0]) + (tx - rmin[0]));
}
// keys of tile >= ntiles (culled pairs, sorted last) are in no range
__global__ __launch_bounds__(256) void k_ranges32(int L, const unsigned* __restrict__ keys, unsigned ntiles,
                                                  uint2* __restrict__ ranges) {
  // each lane compares 4 consecutive keys (one 16-byte load) with their predecessors:
  // a quarter of the load instructions of a lane per key (bicycle: 30M keys)
  const int i0 = 4 * (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i0 >= L) return;
  unsigned k[5];  // k[0]: key i0 - 1
  if (i0 + 4 <= L) {
    const uint4 q = *reinterpret_cast<const uint4*>(keys + i0);
    k[1] = q.x;
    k[2] = q.y;
    k[3] = q.z;
    k[4] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) k[1 + j] = i0 + j < L ? keys[i0 + j] : 0u;
  }
  k[0] = i0 ? keys[i0 - 1] : 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int idx = i0 + j;
    if (idx >= L) break;
    const unsigned cur = k[1 + j] & kTileField;
    const bool live = cur < ntiles;
    if (idx == 0) {
      if (live) ranges[cur].x = 0;
    } else {
      const unsigned prev = k[j] & kTileField;
      if (cur != prev) {
        if (prev < ntiles) ranges[prev].y = idx;
        if (live) ranges[cur].x = idx;
      }
    }
    if (idx == L - 1 && live) ranges[cur].y = L;
  }
}

// ------------------------------------------------------------- backward --
// Per-pixel adjoint of the blend (upstream BACKWARD::renderCUDA), back to
// front.  Pair record (3 x float4 at the pair's emission index):
//   (dmean2D.x, dmean2D.y, dconic.a, dconic.b) (dconic.c, dopacity, dR, dG) (dB, 0, 0, 0)
// with upstream's conventions: dmean2D w.r.t. NDC (x W/2, H/2), the conic's
// off-diagonal term halved, alpha's 0.99 clamp not differentiated.
constexpr int kRec = 9;
#ifndef GSMPM_RBWD_DPP
#define GSMPM_RBWD_DPP 1  // 0: __shfl_xor wave sums (A/B)
#endif


__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// Sum over the wave, valid in lane 63 only: six DPP adds (quad swaps, row
// shifts, row broadcasts) instead of six LDS-crossbar permutes (__shfl_xor is
// ds_bpermute_b32 here).  Lanes whose DPP source is out of range add 0.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_src(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
}
__device__ __forceinline__ float wave_total63(float v) {
  v += dpp_src<0xb1>(v);         // quad_perm [1,0,3,2]
  v += dpp_src<0x4e>(v);         // quad_perm [2,3,0,1]
  v += dpp_src<0x114>(v);        // row_shr:4
  v += dpp_src<0x118>(v);        // row_shr:8
  v += dpp_src<0x142, 0xa>(v);   // row_bcast:15 into rows 1, 3
  v += dpp_src<0x143, 0xc>(v);   // row_bcast:31 into rows 2, 3
  return v;
}

// Test mode (GSMPM_RASTER_POISON=1): every listed pair's record set to NaN
// before k_render_bwd, which must overwrite each one (a record left unwritten
// would otherwise hold whatever the reused buffer held -- the round-1
// 5.98e25 means3D gradients); culled pairs keep the zeros of the memset.
__global__ __launch_bounds__(256) void k_poison_listed(const uint2* __restrict__ ranges,
                                                       const unsigned* __restrict__ pos_sorted,
                                                       float4* __restrict__ rec) {
  const uint2 r = ranges[blockIdx.x];
  const float nan = __int_as_float(0x7fc00000);
  for (unsigned k = r.x + threadIdx.x; k < r.y; k += 256) {
    float4* p = rec + (size_t)pos_sorted[k] * 3;
    p[0] = p[1] = p[2] = make_float4(nan, nan, nan, nan);
  }
}

__global__ __launch_bounds__(kBlock) void k_render_bwd(const uint2* __restrict__ ranges,
                                                       const unsigned* __restrict__ pos_sorted,
                                                       const unsigned* __restrict__ ids, int W, int H, int gx,
                                                       const float2* __restrict__ xy, const float4* __restrict__ conic_o,
                                                       const float4* __restrict__ rgbo, const float* __restrict__ bg,
                                                       const float* __restrict__ final_T,
                                                       const int* __restrict__ n_contrib,
                                                       const float* __restrict__ dL_dpix, float4* __restrict__ rec) {
  __shared__ float2 s_xy[kBlock];
  __shared__ float4 s_co[kBlock];
  __shared__ float4 s_rgb[kBlock];
  __shared__ float s_part[kBlock / 64][kRec][kBlock];
  __shared__ int s_maxlast;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tx = threadIdx.x % kBX, ty = threadIdx.x / kBX;
  const int px = blockIdx.x * kBX + tx, py = blockIdx.y * kBY + ty;
  const bool inside = px < W && py < H;
  const uint2 range = ranges[blockIdx.y * gx + blockIdx.x];
  const int todo0 = (int)(range.y - range.x);
  const size_t pix = (size_t)py * W + px, HW = (size_t)H * W;
  const float T_final = inside ? final_T[pix] : 0.f;
  const int last = inside ? n_contrib[pix] : 0;
  float dpx[3] = {0.f, 0.f, 0.f};
  if (inside)
    for (int ch = 0; ch < 3; ++ch) dpx[ch] = dL_dpix[ch * HW + pix];
  const float bg_dot = bg[0] * dpx[0] + bg[1] * dpx[1] + bg[2] * dpx[2];
  if (threadIdx.x == 0) s_maxlast = 0;
  __syncthreads();
  atomicMax(&s_maxlast, last);
  __syncthreads();
  const int maxlast = s_maxlast;  // list positions >= maxlast contribute to no pixel of the tile
  float T = T_final, accum[3] = {0.f, 0.f, 0.f}, last_color[3] = {0.f, 0.f, 0.f}, last_alpha = 0.f;
  const float pfx = (float)px, pfy = (float)py;
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  const int rounds = (todo0 + kBlock - 1) / kBlock;
  for (int i = 0; i < rounds; ++i) {
    const int hi = todo0 - i * kBlock;          // this batch covers positions [hi - nb, hi)
    const int nb = min(kBlock, hi);
    const int myp = hi - 1 - (int)threadIdx.x;  // list position of this thread's element
    if (hi - nb >= maxlast) {                   // nothing in this batch contributes: zero records
      if ((int)threadIdx.x < nb) {
        float4* r = rec + (size_t)pos_sorted[range.x + myp] * 3;
        r[0] = r[1] = r[2] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      continue;
    }
    __syncthreads();
    if ((int)threadIdx.x < nb) {
      const unsigned id = ids[range.x + myp];
      const float2 gxy = xy[id];
      const float4 gco = conic_o[id];
      s_xy[threadIdx.x] = gxy;
      s_co[threadIdx.x] = gco;
      s_rgb[threadIdx.x] = rgbo[id];
    }
    __syncthreads();
    for (int j = 0; j < nb; ++j) {
      const int contributor = hi - 1 - j;
      float g[kRec] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      bool act = false;
      if (contributor < last) {
        const float2 gp = s_xy[j];
        const float dx = gp.x - pfx, dy = gp.y - pfy;
        const float4 co = s_co[j];
        const float power = __builtin_fmaf(-0.5f, __builtin_fmaf(co.x * dx, dx, co.z * dy * dy), -co.y * dx * dy);
        if (power <= 0.0f) {
          const float G = __builtin_amdgcn_exp2f(power * 1.4426950408889634f);
          const float alpha = fminf(0.99f, co.w * G);
          if (alpha >= 1.0f / 255.0f) {
            act = true;
            T = T / (1.f - alpha);
            const float dchannel_dcolor = alpha * T;
            const float4 c = s_rgb[j];
            const float cc[3] = {c.x, c.y, c.z};
            float dL_dalpha = 0.f;
            for (int ch = 0; ch < 3; ++ch) {
              accum[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum[ch];
              last_color[ch] = cc[ch];
              dL_dalpha += (cc[ch] - accum[ch]) * dpx[ch];
              g[6 + ch] = dchannel_dcolor * dpx[ch];
            }
            dL_dalpha *= T;
            last_alpha = alpha;
            dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
            const float dL_dG = co.w * dL_dalpha;
            const float gdx = G * dx, gdy = G * dy;
            const float dG_ddelx = -gdx * co.x - gdy * co.y;
            const float dG_ddely = -gdy * co.z - gdx * co.y;
            g[0] = dL_dG * dG_ddelx * ddelx_dx;
            g[1] = dL_dG * dG_ddely * ddely_dy;
            g[2] = -0.5f * gdx * dx * dL_dG;
            g[3] = -0.5f * gdx * dy * dL_dG;
            g[4] = -0.5f * gdy * dy * dL_dG;
            g[5] = G * dL_dalpha;
          }
        }
      }
#if GSMPM_RBWD_DPP
      if (__ballot(act)) {
#pragma unroll
        for (int q = 0; q < kRec; ++q) g[q] = wave_total63(g[q]);
      }
      if (lane == 63)
#pragma unroll
        for (int q = 0; q < kRec; ++q) s_part[wave][q][j] = g[q];
#else
      if (__ballot(act)) {
#pragma unroll
        for (int q = 0; q < kRec; ++q) g[q] = wave_sum(g[q]);
      }
      if (lane == 0)
#pragma unroll
        for (int q = 0; q < kRec; ++q) s_part[wave][q][j] = g[q];
#endif
    }
    __syncthreads();
    if ((int)threadIdx.x < nb) {
      const int j = threadIdx.x;
      float o[kRec];
#pragma unroll
      for (int q = 0; q < kRec; ++q) o[q] = s_part[0][q][j] + s_part[1][q][j] + s_part[2][q][j] + s_part[3][q][j];
      float4* r = rec + (size_t)pos_sorted[range.x + myp] * 3;
      r[0] = make_float4(o[0], o[1], o[2], o[3]);
      r[1] = make_float4(o[4], o[5], o[6], o[7]);
      r[2] = make_float4(o[8], 0.f, 0.f, 0.f);
    }
  }
}

__device__ __forceinline__ void dnormvdv(const float v[3], const float dv[3], float out[3]) {
  const float sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
  out[0] = ((sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
  out[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
  out[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

struct RasterGrads {
  float *dmeans2D, *dcolors, *dopacity, *dmeans3D, *dcov3D, *dsh, *dscales, *drot;
};

// computeColorFromSH backward (upstream): dL/dsh and the view-direction term of dL/dmean
__device__ void sh_backward(const RasterDev& a, int idx, const float* pos, unsigned clamp, const float dcol[3],
                            float* dsh, float dmean[3]) {
  const float dir_orig[3] = {pos[0] - a.campos[0], pos[1] - a.campos[1], pos[2] - a.campos[2]};
  const float len = sqrtf(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
  const float x = dir_orig[0] / len, y = dir_orig[1] / len, z = dir_orig[2] / len;
  const float* sh = a.shs + (size_t)idx * a.M * 3;
  float g[3];
  for (int ch = 0; ch < 3; ++ch) g[ch] = ((clamp >> ch) & 1u) ? 0.f : dcol[ch];
  float dRdx[3] = {0.f, 0.f, 0.f}, dRdy[3] = {0.f, 0.f, 0.f}, dRdz[3] = {0.f, 0.f, 0.f};
  const int used = a.D > 2 ? 16 : a.D > 1 ? 9 : a.D > 0 ? 4 : 1;
  float coef[16];
  coef[0] = kSH_C0;
  if (a.D > 0) {
    coef[1] = -kSH_C1 * y;
    coef[2] = kSH_C1 * z;
    coef[3] = -kSH_C1 * x;
    for (int ch = 0; ch < 3; ++ch) {
      dRdx[ch] = -kSH_C1 * sh[3 * 3 + ch];
      dRdy[ch] = -kSH_C1 * sh[1 * 3 + ch];
      dRdz[ch] = kSH_C1 * sh[2 * 3 + ch];
    }
    if (a.D > 1) {
      const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      coef[4] = kSH_C2[0] * xy;
      coef[5] = kSH_C2[1] * yz;
      coef[6] = kSH_C2[2] * (2.f * zz - xx - yy);
      coef[7] = kSH_C2[3] * xz;
      coef[8] = kSH_C2[4] * (xx - yy);
      for (int ch = 0; ch < 3; ++ch) {
        const float* S = sh + ch;
        dRdx[ch] += kSH_C2[0] * y * S[4 * 3] + kSH_C2[2] * 2.f * -x * S[6 * 3] + kSH_C2[3] * z * S[7 * 3] +
                    kSH_C2[4] * 2.f * x * S[8 * 3];
        dRdy[ch] += kSH_C2[0] * x * S[4 * 3] + kSH_C2[1] * z * S[5 * 3] + kSH_C2[2] * 2.f * -y * S[6 * 3] +
                    kSH_C2[4] * 2.f * -y * S[8 * 3];
        dRdz[ch] += kSH_C2[1] * y * S[5 * 3] + kSH_C2[2] * 2.f * 2.f * z * S[6 * 3] + kSH_C2[3] * x * S[7 * 3];
      }
      if (a.D > 2) {
        coef[9] = kSH_C3[0] * y * (3.f * xx - yy);
        coef[10] = kSH_C3[1] * xy * z;
        coef[11] = kSH_C3[2] * y * (4.f * zz - xx - yy);
        coef[12] = kSH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
        coef[13] = kSH_C3[4] * x * (4.f * zz - xx - yy);
        coef[14] = kSH_C3[5] * z * (xx - yy);
        coef[15] = kSH_C3[6] * x * (xx - 3.f * yy);
        for (int ch = 0; ch < 3; ++ch) {
          const float* S = sh + ch;
          dRdx[ch] += kSH_C3[0] * S[9 * 3] * 3.f * 2.f * xy + kSH_C3[1] * S[10 * 3] * yz +
                      kSH_C3[2] * S[11 * 3] * -2.f * xy + kSH_C3[3] * S[12 * 3] * -3.f * 2.f * xz +
                      kSH_C3[4] * S[13 * 3] * (-3.f * xx + 4.f * zz - yy) + kSH_C3[5] * S[14 * 3] * 2.f * xz +
                      kSH_C3[6] * S[15 * 3] * 3.f * (xx - yy);
          dRdy[ch] += kSH_C3[0] * S[9 * 3] * 3.f * (xx - yy) + kSH_C3[1] * S[10 * 3] * xz +
                      kSH_C3[2] * S[11 * 3] * (-3.f * yy + 4.f * zz - xx) + kSH_C3[3] * S[12 * 3] * -3.f * 2.f * yz +
                      kSH_C3[4] * S[13 * 3] * -2.f * xy + kSH_C3[5] * S[14 * 3] * -2.f * yz +
                      kSH_C3[6] * S[15 * 3] * -3.f * 2.f * xy;
          dRdz[ch] += kSH_C3[1] * S[10 * 3] * xy + kSH_C3[2] * S[11 * 3] * 4.f * 2.f * yz +
                      kSH_C3[3] * S[12 * 3] * 3.f * (2.f * zz - xx - yy) + kSH_C3[4] * S[13 * 3] * 4.f * 2.f * xz +
                      kSH_C3[5] * S[14 * 3] * (xx - yy);
        }
      }
    }
  }
  float* d = dsh + (size_t)idx * a.M * 3;
  for (int k = 0; k < a.M; ++k)
    for (int ch = 0; ch < 3; ++ch) d[k * 3 + ch] = k < used ? coef[k] * g[ch] : 0.f;
  const float dL_ddir[3] = {dRdx[0] * g[0] + dRdx[1] * g[1] + dRdx[2] * g[2],
                            dRdy[0] * g[0] + dRdy[1] * g[1] + dRdy[2] * g[2],
                            dRdz[0] * g[0] + dRdz[1] * g[1] + dRdz[2] * g[2]};
  float dm[3];
  dnormvdv(dir_orig, dL_ddir, dm);
  for (int q = 0; q < 3; ++q) dmean[q] += dm[q];
}

// computeCov3D backward: dL/d(mod * scale) and dL/d(unnormalised quaternion)
__device__ void cov3d_backward(const float* s, float mod, const float* rot, const float* dc, float* ds, float* dq) {
  const float S[3] = {mod * s[0], mod * s[1], mod * s[2]};
  const float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
  const float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                      2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                      2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
  const float G[9] = {dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2], 0.5f * dc[4], dc[5]};
  float M[9], dM[9], dR[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[i * 3 + j] = R[i * 3 + j] * S[j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dM[i * 3 + j] = 2.f * (G[i * 3 + 0] * M[0 * 3 + j] + G[i * 3 + 1] * M[1 * 3 + j] + G[i * 3 + 2] * M[2 * 3 + j]);
  for (int j = 0; j < 3; ++j) {
    ds[j] = dM[0 * 3 + j] * R[0 * 3 + j] + dM[1 * 3 + j] * R[1 * 3 + j] + dM[2 * 3 + j] * R[2 * 3 + j];
    for (int i = 0; i < 3; ++i) dR[i * 3 + j] = dM[i * 3 + j] * S[j];
  }
  dq[0] = 2.f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
  dq[1] = 2.f * (y * dR[1] + z * dR[2] + y * dR[3] - 2.f * x * dR[4] - r * dR[5] + z * dR[6] + r * dR[7] - 2.f * x * dR[8]);
  dq[2] = 2.f * (-2.f * y * dR[0] + x * dR[1] + r * dR[2] + x * dR[3] + z * dR[5] - r * dR[6] + z * dR[7] - 2.f * y * dR[8]);
  dq[3] = 2.f * (-2.f * z * dR[0] - r * dR[1] + x * dR[2] + r * dR[3] - 2.f * z * dR[4] + y * dR[5] + x * dR[6] + y * dR[7]);
}

// computeCov2DCUDA + preprocessCUDA backward, one lane per Gaussian.
__global__ __launch_bounds__(256) void k_preprocess_bwd(RasterDev a, const int* __restrict__ radii,
                                                        const unsigned* __restrict__ offsets,
                                                        const float4* __restrict__ rgbo, const float4* __restrict__ rec,
                                                        RasterGrads o) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.P) return;
  float g[kRec] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dm[3] = {0.f, 0.f, 0.f}, dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool on = radii[idx] > 0;
  const float* m = a.means3D + (size_t)idx * 3;
  float c6[6];
  const float* c3 = nullptr;
  if (on) {
    const unsigned b = idx ? offsets[idx - 1] : 0u, e = offsets[idx];
    for (unsigned k = b; k < e; ++k) {
      const float4 r0 = rec[(size_t)k * 3], r1 = rec[(size_t)k * 3 + 1], r2 = rec[(size_t)k * 3 + 2];
      g[0] += r0.x; g[1] += r0.y; g[2] += r0.z; g[3] += r0.w;
      g[4] += r1.x; g[5] += r1.y; g[6] += r1.z; g[7] += r1.w;
      g[8] += r2.x;
    }
    if (a.cov3D_precomp) {
      c3 = a.cov3D_precomp + (size_t)idx * 6;
    } else {
      cov3d_from_sr(a.scales + (size_t)idx * 3, a.scale_modifier, a.rotations + (size_t)idx * 4, c6);
      c3 = c6;
    }
    const float* vm = a.viewmatrix;
    float t[3];
    xform4x3(m, vm, t);
    const float limx = 1.3f * a.tanfovx, limy = 1.3f * a.tanfovy;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    const float x_mul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    const float y_mul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const float hx = a.focal_x, hy = a.focal_y;
    const float J00 = hx / t[2], J02 = -(hx * t[0]) / (t[2] * t[2]);
    const float J11 = hy / t[2], J12 = -(hy * t[1]) / (t[2] * t[2]);
    const float Wm[9] = {vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]};
    float T0[3], T1[3];
    for (int c = 0; c < 3; ++c) {
      T0[c] = J00 * Wm[0 * 3 + c] + J02 * Wm[2 * 3 + c];
      T1[c] = J11 * Wm[1 * 3 + c] + J12 * Wm[2 * 3 + c];
    }
    const float V[9] = {c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]};
    float VT0[3], VT1[3];
    for (int r = 0; r < 3; ++r) {
      VT0[r] = V[r * 3 + 0] * T0[0] + V[r * 3 + 1] * T0[1] + V[r * 3 + 2] * T0[2];
      VT1[r] = V[r * 3 + 0] * T1[0] + V[r * 3 + 1] * T1[1] + V[r * 3 + 2] * T1[2];
    }
    const float ca = T0[0] * VT0[0] + T0[1] * VT0[1] + T0[2] * VT0[2] + 0.3f;
    const float cb = T0[0] * VT1[0] + T0[1] * VT1[1] + T0[2] * VT1[2];
    const float cc = T1[0] * VT1[0] + T1[1] * VT1[1] + T1[2] * VT1[2] + 0.3f;
    const float denom = ca * cc - cb * cb;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float dco[3] = {g[2], g[3], g[4]};
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    if (denom2inv != 0.f) {
      dL_da = denom2inv * (-cc * cc * dco[0] + 2.f * cb * cc * dco[1] + (denom - ca * cc) * dco[2]);
      dL_dc = denom2inv * (-ca * ca * dco[2] + 2.f * ca * cb * dco[1] + (denom - ca * cc) * dco[0]);
      dL_db = denom2inv * 2.f * (cb * cc * dco[0] - (denom + 2.f * cb * cb) * dco[1] + ca * cb * dco[2]);
      const int di[6] = {0, 0, 0, 1, 1, 2}, dj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
      for (int e2 = 0; e2 < 6; ++e2) {
        const int p = di[e2], q = dj[e2];
        dcov[e2] = p == q ? T0[p] * T0[p] * dL_da + T0[p] * T1[p] * dL_db + T1[p] * T1[p] * dL_dc
                          : 2.f * T0[p] * T0[q] * dL_da + (T0[p] * T1[q] + T0[q] * T1[p]) * dL_db +
                                2.f * T1[p] * T1[q] * dL_dc;
      }
    }
    float dT0[3], dT1[3];
    for (int c = 0; c < 3; ++c) {
      dT0[c] = 2.f * VT0[c] * dL_da + VT1[c] * dL_db;
      dT1[c] = VT0[c] * dL_db + 2.f * VT1[c] * dL_dc;
    }
    const float dJ00 = Wm[0] * dT0[0] + Wm[1] * dT0[1] + Wm[2] * dT0[2];
    const float dJ02 = Wm[6] * dT0[0] + Wm[7] * dT0[1] + Wm[8] * dT0[2];
    const float dJ11 = Wm[3] * dT1[0] + Wm[4] * dT1[1] + Wm[5] * dT1[2];
    const float dJ12 = Wm[6] * dT1[0] + Wm[7] * dT1[1] + Wm[8] * dT1[2];
    const float tz = 1.f / t[2], tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = x_mul * -hx * tz2 * dJ02;
    const float dty = y_mul * -hy * tz2 * dJ12;
    const float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2.f * hx * t[0]) * tz3 * dJ02 + (2.f * hy * t[1]) * tz3 * dJ12;
    dm[0] = vm[0] * dtx + vm[1] * dty + vm[2] * dtz;
    dm[1] = vm[4] * dtx + vm[5] * dty + vm[6] * dtz;
    dm[2] = vm[8] * dtx + vm[9] * dty + vm[10] * dtz;
    const float* pm = a.projmatrix;
    const float hw = pm[3] * m[0] + pm[7] * m[1] + pm[11] * m[2] + pm[15];
    const float mw = 1.0f / (hw + 0.0000001f);
    const float mul1 = (pm[0] * m[0] + pm[4] * m[1] + pm[8] * m[2] + pm[12]) * mw * mw;
    const float mul2 = (pm[1] * m[0] + pm[5] * m[1] + pm[9] * m[2] + pm[13]) * mw * mw;
    dm[0] += (pm[0] * mw - pm[3] * mul1) * g[0] + (pm[1] * mw - pm[3] * mul2) * g[1];
    dm[1] += (pm[4] * mw - pm[7] * mul1) * g[0] + (pm[5] * mw - pm[7] * mul2) * g[1];
    dm[2] += (pm[8] * mw - pm[11] * mul1) * g[0] + (pm[9] * mw - pm[11] * mul2) * g[1];
  }
  if (a.shs) {
    if (on) {
      sh_backward(a, idx, m, __float_as_uint(rgbo[idx].w), g + 6, o.dsh, dm);
    } else {
      float* d = o.dsh + (size_t)idx * a.M * 3;
      for (int k = 0; k < a.M * 3; ++k) d[k] = 0.f;
    }
  }
  if (a.scales) {
    float ds[3] = {0.f, 0.f, 0.f}, dq[4] = {0.f, 0.f, 0.f, 0.f};
    if (on) cov3d_backward(a.scales + (size_t)idx * 3, a.scale_modifier, a.rotations + (size_t)idx * 4, dcov, ds, dq);
    for (int q = 0; q < 3; ++q) o.dscales[(size_t)idx * 3 + q] = ds[q];
    for (int q = 0; q < 4; ++q) o.drot[(size_t)idx * 4 + q] = dq[q];
  }
  o.dmeans2D[(size_t)idx * 3 + 0] = g[0];
  o.dmeans2D[(size_t)idx * 3 + 1] = g[1];
  o.dmeans2D[(size_t)idx * 3 + 2] = 0.f;
  for (int q = 0; q < 3; ++q) {
    o.dcolors[(size_t)idx * 3 + q] = g[6 + q];
    o.dmeans3D[(size_t)idx * 3 + q] = dm[q];
  }
  o.dopacity[idx] = g[5];
  for (int q = 0; q < 6; ++q) o.dcov3D[(size_t)idx * 6 + q] = dcov[q];
}

__global__ __launch_bounds__(256) void k_mark_visible(const float* __restrict__ m, int P, const float* __restrict__ vm,
                                                      uint8_t* __restrict__ vis) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= P) return;
  float pv[3];
  xform4x3(m + (size_t)idx * 3, vm, pv);
  vis[idx] = pv[2] > 0.2f ? 1 : 0;
}

static int msb_bits(unsigned n) {
  int b = 0;
  while (n > 0) {
    ++b;
    n >>= 1;
  }
  return b;
}

}  // namespace gsmpm

using namespace gsmpm;

struct gsmpm_raster {
  // per-Gaussian buffers
  size_t capP = 0;
  int* radii_tmp = nullptr;
  float* depth = nullptr;
  float2* xy = nullptr;
  float4* conic = nullptr;
  float4* rgb = nullptr;
  unsigned long long* tiles = nullptr;  // (3-sigma tile count << 32) | binned tile count
  uint2* rect = nullptr;                // binned tile rect (pack_rect)
  unsigned* offsets = nullptr;
  void* scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  // binning buffers
  size_t capK = 0;
  unsigned long long *keys = nullptr, *keys_sorted = nullptr;
  unsigned *vals = nullptr, *vals_sorted = nullptr;
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  unsigned* ids_sorted = nullptr;  // Gaussian id per sorted pair (vals_sorted holds emission indices)
  unsigned* estart = nullptr;      // [capK / kEmitT + 2] k_emit_starts
  unsigned *dorder = nullptr, *dsorted = nullptr;  // [capP] depth order
  unsigned long long* offr = nullptr;  // [capP] inclusive scan of tiles in depth order (index order: upstream keys)
  void* dsort_tmp = nullptr;
  unsigned* hist = nullptr;  // [2 * capH] tile-major chunk histogram, then its exclusive scan
  size_t capH = 0;
  size_t dsort_tmp_bytes = 0;
  bool slots_pending = false;
  bool offsets_pending = false;  // depth-ordered forward: the index-order tile scan (offsets) is left to the backward
  bool emit_culled = false;  // the tile lists omit culled pairs: their records must read zero  // vals_sorted still to be derived (depth-ordered path)
  float4* rec = nullptr;           // backward pair records, 3 x float4 per pair
  size_t capRec = 0;
  // tile ranges
  size_t capT = 0;
  uint2* ranges = nullptr;
  int* dsort_tl = nullptr;  // [2 + 2 * capT] k_tile_dsort's size-class lists
  unsigned* h_count = nullptr;  // [4] pinned, mapped + coherent (the device writes K, num_rendered, overflow, big-bucket flag)
  // the hand-written depth order (dsort.h): state + bucket arrays (fixed size), per-Gaussian runs
  char* ds_state = nullptr;    // kDsStateBytes, zero when idle
  unsigned *ds_bbase = nullptr, *ds_bcur = nullptr, *ds_blist = nullptr, *ds_bbig = nullptr;  // [kDsNBMax]
  unsigned long long* ds_bpre = nullptr;  // [kDsNBMax]
  unsigned *ds_key = nullptr, *ds_val = nullptr;  // [capP]
  unsigned* ttot = nullptr;    // [capT + 2] chunked tile sort: tile totals (k_tile_rows)
  unsigned long long* scan_bt = nullptr;  // [capP / 1024 + 1] block totals of the index-order scans (scan.h)
  unsigned* dl_h = nullptr;    // [2 * 256 * (capP / kDlChunk + 1) + 256] the LSD depth order's counts, prefixes, totals
  long dsort_fallbacks = 0;    // forwards whose depth order fell back to the library sort
  // the async form (gsmpm_raster_forward_async): pair buffers carved for async_cap
  // pairs, the counts published to async_counts, no host synchronisation
  int64_t async_cap = 0;
  unsigned* async_counts = nullptr;
  hipEvent_t count_ev = nullptr;  // recorded after the publishing kernels: surfaces a fault while the host spins
  // per pixel (backward)
  size_t capPix = 0;
  float* final_T = nullptr;
  int* n_contrib = nullptr;
  // the forward the state belongs to
  int P = -1, W = 0, H = 0, gx = 0, gy = 0;
  unsigned K = 0, K_full = 0;  // binned pairs, num_rendered
  bool forward_only = false;  // gsmpm_raster_set_forward_only: no per-pixel state for a backward
  bool has_pixel_state = false;
  // caller-owned workspace (gsmpm_raster_forward_ws): every buffer is carved
  // from it, nothing is allocated; the pair-dependent part is carved once the
  // pair count is known (ws_carve_pairs), or the call fails with GSMPM_ESPACE
  char* ws = nullptr;
  size_t ws_bytes = 0, ws_pre = 0;  // workspace size, bytes of the pair-independent part
  int64_t pairs_needed = 0;
};

static DsortBufs dsort_bufs(gsmpm_raster* r) {
  DsortBufs d;
  d.st = reinterpret_cast<unsigned*>(r->ds_state);
  d.bcount = d.st ? d.st + kDsWords : nullptr;
  d.bsum = d.st ? reinterpret_cast<unsigned long long*>(d.bcount + kDsNBMax) : nullptr;
  d.bbase = r->ds_bbase;
  d.bcur = r->ds_bcur;
  d.bpre = r->ds_bpre;
  d.blist = r->ds_blist;
  d.bbig = r->ds_bbig;
  d.dkey = r->ds_key;
  d.dval = r->ds_val;
  d.bts = d.st ? reinterpret_cast<unsigned long long*>(d.bsum + kDsNBMax) : nullptr;
  d.btc = d.st ? reinterpret_cast<unsigned*>(d.bts + kDsNBMax / kDsBlk) : nullptr;
  d.shard = d.st ? reinterpret_cast<unsigned*>(r->ds_state + kDsShardOff) : nullptr;
  return d;
}
static size_t dl_h_words(size_t cap) { return 2 * 256 * (cap / kDlChunk + 1) + 256; }
static DlBufs dl_bufs(gsmpm_raster* r, int P) {
  const size_t nch = (size_t)div_up(P, kDlChunk);
  DlBufs b;
  b.st = reinterpret_cast<unsigned*>(r->ds_state);
  b.shard = reinterpret_cast<unsigned*>(r->ds_state + kDsShardOff);
  b.k0 = r->ds_key;
  b.v0 = r->ds_val;
  b.k1 = r->dsorted;
  b.v1 = r->dorder;  // free until the final scan writes the order (in place when it is the last pass's)
  b.H = r->dl_h;
  b.Hs = r->dl_h + 256 * nch;
  b.tot = r->dl_h + 2 * 256 * nch;
  return b;
}
// buckets of the depth order: a power of two, ~8 visible Gaussians a bucket, in [1024, kDsNBMax]
static int dsort_buckets(int P) {
  int nb = 1024;
  while (nb < kDsNBMax && nb * 8 < P) nb <<= 1;
  return nb;
}

// inclusive scan of the tiles words in Gaussian-index order (scan.h): T = unsigned
// for the binned count alone, unsigned long long for both counts
template <typename T>
static void scan_tiles(gsmpm_raster* r, int P, T* out, hipStream_t st) {
  const int nb = div_up(P, kScanBlk);
  T* bt = reinterpret_cast<T*>(r->scan_bt);
  hipLaunchKernelGGL(k_scan_blocks<T>, dim3(nb), dim3(256), 0, st, (const unsigned long long*)r->tiles, P, bt);
  hipLaunchKernelGGL(k_scan_apply<T>, dim3(nb), dim3(256), 0, st, (const unsigned long long*)r->tiles, P,
                     (const T*)bt, out);
}

static int grow(void** p, size_t bytes) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  GSMPM_HIP(hipMalloc(p, bytes ? bytes : 16));
  return GSMPM_OK;
}

// ---- caller-owned workspace ----
// Layout: the pair-independent buffers (per Gaussian, per tile, the device
// scan / depth-sort temporaries), then the pair buffers for `pairs` binned
// pairs (keys, values, emission starts, chunk histograms, the tile-sort
// temporary: the largest any binning path takes), each 256-B aligned.  A
// walk over the buffers in a fixed order gives both the size and, with a
// base, the pointers.
struct WsWalk {
  char* base;
  size_t off = 0;
  template <class T>
  void take(T*& p, size_t bytes) {
    off = (off + 255) & ~size_t(255);
    if (base) p = reinterpret_cast<T*>(base + off);
    off += std::max<size_t>(bytes, 16);
  }
};
static int ws_pre_walk(WsWalk& w, gsmpm_raster* r, size_t P, size_t ntiles) {
  const size_t cap = std::max<size_t>(P, 1);
  size_t dbytes = 0, obytes = 0, sbytes = 0, gbytes = 0, ibytes = 0;
  GSMPM_HIP(rocprim::radix_sort_pairs(nullptr, dbytes, reinterpret_cast<unsigned*>(r->depth), r->dsorted,
                                      rocprim::counting_iterator<unsigned>(0u), r->dorder, cap, 0, 32, hipStream_t(0)));
  if (kDepthOnesweepMin > 0 && cap >= kDepthOnesweepMin)
    GSMPM_HIP(rocprim::radix_sort_pairs<OnesweepSort>(nullptr, obytes, reinterpret_cast<unsigned*>(r->depth),
                                                      r->dsorted, rocprim::counting_iterator<unsigned>(0u), r->dorder,
                                                      cap, 0, 32, hipStream_t(0)));
  GSMPM_HIP(rocprim::inclusive_scan(nullptr, sbytes, binned_tiles(r->tiles), r->offsets, cap,
                                    rocprim::plus<unsigned>(), hipStream_t(0)));
  GSMPM_HIP(rocprim::inclusive_scan(nullptr, gbytes, ranked_tiles(r->dorder, r->tiles), r->offr, cap,
                                    rocprim::plus<unsigned long long>(), hipStream_t(0)));
  GSMPM_HIP(rocprim::inclusive_scan(nullptr, ibytes, r->tiles, r->offr, cap, rocprim::plus<unsigned long long>(),
                                    hipStream_t(0)));
  r->dsort_tmp_bytes = std::max(dbytes, obytes);
  r->scan_tmp_bytes = std::max(sbytes, std::max(gbytes, ibytes));
  w.take(r->ds_state, kDsStateBytes);  // first, at a fixed offset: zero when idle (the caller zero-fills once)
  w.take(r->ds_bbase, kDsNBMax * sizeof(unsigned));
  w.take(r->ds_bcur, kDsNBMax * sizeof(unsigned));
  w.take(r->ds_blist, kDsNBMax * sizeof(unsigned));
  w.take(r->ds_bbig, kDsNBMax * sizeof(unsigned));
  w.take(r->ds_bpre, kDsNBMax * sizeof(unsigned long long));
  w.take(r->ds_key, cap * sizeof(unsigned));
  w.take(r->ds_val, cap * sizeof(unsigned));
  w.take(r->ttot, (ntiles + 2) * sizeof(unsigned));
  w.take(r->scan_bt, (cap / kScanBlk + 1) * sizeof(unsigned long long));
  w.take(r->dl_h, dl_h_words(cap) * sizeof(unsigned));
  w.take(r->depth, cap * sizeof(float));
  w.take(r->xy, cap * sizeof(float2));
  w.take(r->conic, cap * sizeof(float4));
  w.take(r->rgb, cap * sizeof(float4));
  w.take(r->tiles, cap * sizeof(unsigned long long));
  w.take(r->rect, cap * sizeof(uint2));
  w.take(r->offsets, cap * sizeof(unsigned));
  w.take(r->dorder, cap * sizeof(unsigned));
  w.take(r->dsorted, cap * sizeof(unsigned));
  w.take(r->offr, cap * sizeof(unsigned long long));
  w.take(r->dsort_tmp, r->dsort_tmp_bytes);
  w.take(r->scan_tmp, r->scan_tmp_bytes);
  w.take(r->ranges, ntiles * sizeof(uint2));
  w.take(r->dsort_tl, (2 + 2 * ntiles) * sizeof(int));
  r->capP = cap;
  r->capT = ntiles;
  return GSMPM_OK;
}
static int ws_pairs_walk(WsWalk& w, gsmpm_raster* r, size_t K, size_t ntiles) {
  const size_t cap = std::max<size_t>(K, 1);
  const int bits = msb_bits((unsigned)ntiles);
  const size_t nch = div_up(cap, (size_t)kChunk);
  const size_t capH = std::max((ntiles + 1) * nch, 256 * nch);
  size_t b[4] = {0, 0, 0, 0};
  GSMPM_HIP(rocprim::radix_sort_pairs(nullptr, b[0], r->keys, r->keys_sorted, rocprim::counting_iterator<unsigned>(0u),
                                      r->vals_sorted, cap, 0, 64, hipStream_t(0)));
  GSMPM_HIP(rocprim::radix_sort_pairs<OnesweepSort>(nullptr, b[1], reinterpret_cast<unsigned*>(r->keys),
                                                    reinterpret_cast<unsigned*>(r->keys_sorted), r->vals,
                                                    r->ids_sorted, cap, 0, bits, hipStream_t(0)));
  GSMPM_HIP(rocprim::exclusive_scan(nullptr, b[2], r->hist, r->hist + capH, 0u, capH, rocprim::plus<unsigned>(),
                                    hipStream_t(0)));
  r->sort_tmp_bytes = std::max(std::max(b[0], b[1]), b[2]);
  w.take(r->keys, cap * 8);
  w.take(r->keys_sorted, cap * 8);
  w.take(r->vals, cap * 4);
  w.take(r->vals_sorted, cap * 4);
  w.take(r->ids_sorted, cap * 4);
  w.take(r->estart, (cap / kEmitT + 2) * 4);
  w.take(r->hist, 2 * capH * sizeof(unsigned));
  w.take(r->sort_tmp, r->sort_tmp_bytes);
  r->capK = cap;
  r->capH = capH;
  return GSMPM_OK;
}
// carve the pair buffers for K pairs from r's workspace, or GSMPM_ESPACE (pairs_needed = K)
static int ws_carve_pairs(gsmpm_raster* r, size_t K, size_t ntiles) {
  WsWalk probe{nullptr, r->ws_pre};
  gsmpm_raster tmp;
  int rc = ws_pairs_walk(probe, &tmp, K, ntiles);
  if (rc) return rc;
  if (probe.off > r->ws_bytes) {
    r->pairs_needed = (int64_t)K;
    set_error("gsmpm_raster_forward_ws: the workspace holds too few pairs for this frame (" + std::to_string(K) +
              " binned pairs need " + std::to_string(probe.off) + " bytes, the workspace has " +
              std::to_string(r->ws_bytes) + "); grow it (gsmpm_raster_workspace_size) and call again");
    return GSMPM_ESPACE;
  }
  WsWalk w{r->ws, r->ws_pre};
  return ws_pairs_walk(w, r, K, ntiles);
}

extern "C" {

int gsmpm_raster_create(gsmpm_raster** out) {
  GSMPM_REQUIRE(out, "gsmpm_raster_create: null argument");
  auto* r = new gsmpm_raster();
  hipError_t e = hipHostMalloc((void**)&r->h_count, 4 * sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&r->count_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc((void**)&r->ds_state, kDsStateBytes);
  if (e == hipSuccess) e = hipMemset(r->ds_state, 0, kDsStateBytes);
  for (unsigned** q : {&r->ds_bbase, &r->ds_bcur, &r->ds_blist, &r->ds_bbig})
    if (e == hipSuccess) e = hipMalloc((void**)q, kDsNBMax * sizeof(unsigned));
  if (e == hipSuccess) e = hipMalloc((void**)&r->ds_bpre, kDsNBMax * sizeof(unsigned long long));
  if (e != hipSuccess) {
    if (r->h_count) (void)hipHostFree(r->h_count);
    if (r->count_ev) (void)hipEventDestroy(r->count_ev);
    for (void* q : {(void*)r->ds_state, (void*)r->ds_bbase, (void*)r->ds_bcur, (void*)r->ds_blist, (void*)r->ds_bbig,
                    (void*)r->ds_bpre})
      if (q) (void)hipFree(q);
    delete r;
    set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
    return GSMPM_EHIP;
  }
  *out = r;
  return GSMPM_OK;
}

int gsmpm_raster_destroy(gsmpm_raster* r) {
  if (!r) return GSMPM_OK;
  for (void* p : {(void*)r->radii_tmp, (void*)r->depth, (void*)r->xy, (void*)r->conic, (void*)r->rgb, (void*)r->tiles, (void*)r->rect,
                  (void*)r->offsets, r->scan_tmp, (void*)r->keys, (void*)r->keys_sorted, (void*)r->vals,
                  (void*)r->vals_sorted, r->sort_tmp, (void*)r->ranges, (void*)r->ids_sorted, (void*)r->estart, (void*)r->rec,
                  (void*)r->final_T, (void*)r->n_contrib, (void*)r->dorder, (void*)r->dsorted, (void*)r->offr, r->dsort_tmp, (void*)r->hist,
                  (void*)r->dsort_tl, (void*)r->ds_state, (void*)r->ds_bbase, (void*)r->ds_bcur, (void*)r->ds_blist,
                  (void*)r->ds_bbig, (void*)r->ds_bpre, (void*)r->ds_key, (void*)r->ds_val, (void*)r->ttot,
                  (void*)r->scan_bt, (void*)r->dl_h})
    if (p) (void)hipFree(p);
  if (r->h_count) (void)hipHostFree(r->h_count);
  if (r->count_ev) (void)hipEventDestroy(r->count_ev);
  delete r;
  return GSMPM_OK;
}

// In-frame timing of the forwards (gsmpm_raster_set_timing): three events per
// forward on its own stream -- at entry, before and after k_render -- so a
// caller can read what k_render and the whole forward took inside a running
// frame loop (beside the simulator) without a host wait in the loop.
// Forwards issued while their stream is being captured are not timed.
// The pending list is bounded: past kTmCap entries a new one first folds the
// oldest completed entries into running sums (a hipEventQuery, never a wait),
// so a caller that turns timing on and never reads it holds at most kTmCap
// forwards' events.  Timing off costs one relaxed atomic load per forward.
namespace {
struct FwdTiming {
  hipEvent_t e[3];
};
constexpr size_t kTmCap = 256;
std::mutex g_tm_mu;
std::atomic<bool> g_tm_on{false};
std::vector<FwdTiming> g_tm_pending, g_tm_free;
double g_tm_kr = 0.0, g_tm_fw = 0.0;  // folded entries' sums (under g_tm_mu)
int64_t g_tm_n = 0;
// fold the oldest completed pending entries (caller holds g_tm_mu)
void tm_fold_locked() {
  size_t k = 0;
  while (k < g_tm_pending.size() && g_tm_pending.size() - k > kTmCap / 2) {
    FwdTiming& t = g_tm_pending[k];
    if (hipEventQuery(t.e[2]) != hipSuccess) break;  // not done yet (in order on one stream)
    float a = 0.f, b = 0.f;
    if (hipEventElapsedTime(&a, t.e[1], t.e[2]) == hipSuccess && hipEventElapsedTime(&b, t.e[0], t.e[2]) == hipSuccess) {
      g_tm_kr += a;
      g_tm_fw += b;
      ++g_tm_n;
    }
    g_tm_free.push_back(t);
    ++k;
  }
  g_tm_pending.erase(g_tm_pending.begin(), g_tm_pending.begin() + (long)k);
}
struct TimingGuard {
  FwdTiming t{};
  bool on = false, done = false;
  hipStream_t st = nullptr;
  explicit TimingGuard(hipStream_t s) : st(s) {
    if (!g_tm_on.load(std::memory_order_relaxed)) return;
    {
      std::lock_guard<std::mutex> lk(g_tm_mu);
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
      if (!g_tm_free.empty()) {
        t = g_tm_free.back();
        g_tm_free.pop_back();
      } else {
        for (auto& e : t.e)
          if (hipEventCreate(&e) != hipSuccess) return;
      }
    }
    on = hipEventRecord(t.e[0], st) == hipSuccess;
  }
  void mark(int i) {
    if (on) on = hipEventRecord(t.e[i], st) == hipSuccess;
    if (on && i == 2) done = true;
  }
  ~TimingGuard() {
    if (t.e[0] == nullptr) return;
    std::lock_guard<std::mutex> lk(g_tm_mu);
    if (done && g_tm_pending.size() >= kTmCap) tm_fold_locked();
    (done ? g_tm_pending : g_tm_free).push_back(t);
  }
};
}  // namespace

int gsmpm_raster_set_timing(int32_t on) {
  g_tm_on.store(on != 0, std::memory_order_relaxed);
  return GSMPM_OK;
}

int gsmpm_raster_timing(double* k_render_ms, double* forward_ms, int64_t* forwards) {
  GSMPM_REQUIRE(k_render_ms && forward_ms && forwards, "gsmpm_raster_timing: null argument");
  std::vector<FwdTiming> got;
  double kr = 0.0, fw = 0.0;
  int64_t n0 = 0;
  {
    std::lock_guard<std::mutex> lk(g_tm_mu);
    got.swap(g_tm_pending);
    kr = g_tm_kr;
    fw = g_tm_fw;
    n0 = g_tm_n;
    g_tm_kr = g_tm_fw = 0.0;
    g_tm_n = 0;
  }
  int rc = GSMPM_OK;
  for (auto& t : got) {
    float a = 0.f, b = 0.f;
    if (rc == GSMPM_OK && (hipEventSynchronize(t.e[2]) != hipSuccess || hipEventElapsedTime(&a, t.e[1], t.e[2]) != hipSuccess ||
                           hipEventElapsedTime(&b, t.e[0], t.e[2]) != hipSuccess)) {
      set_error("gsmpm_raster_timing: event query failed");
      rc = GSMPM_EHIP;
    }
    kr += a;
    fw += b;
  }
  {
    std::lock_guard<std::mutex> lk(g_tm_mu);
    for (auto& t : got) g_tm_free.push_back(t);
  }
  *k_render_ms = kr;
  *forward_ms = fw;
  *forwards = n0 + (int64_t)got.size();
  return rc;
}

int gsmpm_raster_forward(gsmpm_raster* r, const gsmpm_raster_args* in, float* out_color, int32_t* out_radii,
                         int32_t* num_rendered, void* stream) {
  GSMPM_REQUIRE(r && in && out_color && out_radii, "gsmpm_raster_forward: null argument");
  GSMPM_REQUIRE(in->P >= 0 && in->W > 0 && in->H > 0, "gsmpm_raster_forward: bad sizes");
  GSMPM_REQUIRE((in->shs != nullptr) != (in->colors_precomp != nullptr),
                "Please provide excatly one of either SHs or precomputed colors!");
  GSMPM_REQUIRE((in->cov3D_precomp != nullptr) != (in->scales != nullptr && in->rotations != nullptr),
                "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
  GSMPM_REQUIRE(in->means3D && in->opacities && in->viewmatrix && in->projmatrix && in->campos && in->bg,
                "gsmpm_raster_forward: null tensor");
  GSMPM_REQUIRE(in->shs == nullptr || in->M >= 1, "gsmpm_raster_forward: shs needs M >= 1");
  GSMPM_REQUIRE(in->shs == nullptr || in->D < 1 || in->M >= (in->D + 1) * (in->D + 1),
                "gsmpm_raster_forward: too few SH coefficients for sh_degree");
  GSMPM_REQUIRE(!in->prefiltered, "gsmpm_raster_forward: prefiltered=True is not supported (upstream traps too)");
  hipStream_t st = (hipStream_t)stream;
  TimingGuard tmg(st);
  RasterDev a;
  a.P = in->P;
  a.D = in->D;
  a.M = in->M;
  a.W = in->W;
  a.H = in->H;
  a.means3D = in->means3D;
  a.shs = in->shs;
  a.colors_precomp = in->colors_precomp;
  a.opacities = in->opacities;
  a.scales = in->scales;
  a.rotations = in->rotations;
  a.cov3D_precomp = in->cov3D_precomp;
  a.scale_modifier = in->scale_modifier;
  a.viewmatrix = in->viewmatrix;
  a.projmatrix = in->projmatrix;
  a.campos = in->campos;
  a.bg = in->bg;
  a.tanfovx = in->tanfovx;
  a.tanfovy = in->tanfovy;
  a.focal_x = in->W / (2.0f * in->tanfovx);
  a.focal_y = in->H / (2.0f * in->tanfovy);
  a.grid_x = (in->W + kBX - 1) / kBX;
  a.grid_y = (in->H + kBY - 1) / kBY;
  const int P = in->P;
  const size_t ntiles = (size_t)a.grid_x * a.grid_y;
  if (!r->ws && ((size_t)P > r->capP || r->capP == 0)) {
    const size_t cap = std::max<size_t>(P, 1024);
    int rc;
    if ((rc = grow((void**)&r->depth, cap * sizeof(float)))) return rc;
    if ((rc = grow((void**)&r->xy, cap * sizeof(float2)))) return rc;
    if ((rc = grow((void**)&r->conic, cap * sizeof(float4)))) return rc;
    if ((rc = grow((void**)&r->rgb, cap * sizeof(float4)))) return rc;
    if ((rc = grow((void**)&r->tiles, cap * sizeof(unsigned long long)))) return rc;
    if ((rc = grow((void**)&r->rect, cap * sizeof(uint2)))) return rc;
    if ((rc = grow((void**)&r->offsets, cap * sizeof(unsigned)))) return rc;
    if ((rc = grow((void**)&r->dorder, cap * sizeof(unsigned)))) return rc;
    if ((rc = grow((void**)&r->dsorted, cap * sizeof(unsigned)))) return rc;
    if ((rc = grow((void**)&r->offr, cap * sizeof(unsigned long long)))) return rc;
    if ((rc = grow((void**)&r->ds_key, cap * sizeof(unsigned)))) return rc;
    if ((rc = grow((void**)&r->ds_val, cap * sizeof(unsigned)))) return rc;
    if ((rc = grow((void**)&r->scan_bt, (cap / kScanBlk + 1) * sizeof(unsigned long long)))) return rc;
    if ((rc = grow((void**)&r->dl_h, dl_h_words(cap) * sizeof(unsigned)))) return rc;
    size_t bytes = 0, obytes = 0;
    GSMPM_HIP(rocprim::radix_sort_pairs(nullptr, bytes, reinterpret_cast<unsigned*>(r->depth), r->dsorted,
                                                      rocprim::counting_iterator<unsigned>(0u), r->dorder, cap, 0, 32,
                                                      st));
    if (kDepthOnesweepMin > 0 && cap >= kDepthOnesweepMin)
      GSMPM_HIP(rocprim::radix_sort_pairs<OnesweepSort>(nullptr, obytes, reinterpret_cast<unsigned*>(r->depth),
                                                        r->dsorted, rocprim::counting_iterator<unsigned>(0u),
                                                        r->dorder, cap, 0, 32, st));
    bytes = std::max(bytes, obytes);
    if ((rc = grow(&r->dsort_tmp, bytes))) return rc;
    r->dsort_tmp_bytes = bytes;
    bytes = 0;
    GSMPM_HIP(rocprim::inclusive_scan(nullptr, bytes, binned_tiles(r->tiles), r->offsets, cap,
                                      rocprim::plus<unsigned>(), st));
    size_t gbytes = 0, ibytes = 0;
    GSMPM_HIP(rocprim::inclusive_scan(nullptr, gbytes, ranked_tiles(r->dorder, r->tiles), r->offr, cap,
                                      rocprim::plus<unsigned long long>(), st));
    GSMPM_HIP(rocprim::inclusive_scan(nullptr, ibytes, r->tiles, r->offr, cap, rocprim::plus<unsigned long long>(),
                                      st));
    bytes = std::max(bytes, std::max(gbytes, ibytes));
    if ((rc = grow(&r->scan_tmp, bytes))) return rc;
    r->scan_tmp_bytes = bytes;
    r->capP = cap;
  }
  if (!r->ws && ntiles > r->capT) {
    int rc;
    if ((rc = grow((void**)&r->ranges, ntiles * sizeof(uint2)))) return rc;
    if ((rc = grow((void**)&r->dsort_tl, (2 + 2 * ntiles) * sizeof(int)))) return rc;
    if ((rc = grow((void**)&r->ttot, (2 + ntiles) * sizeof(unsigned)))) return rc;
    r->capT = ntiles;
  }
  // tile ranges: the chunked tile sort writes every tile's; the other paths
  // (and K = 0) start from empty ranges
  bool ranges_written = false;
  const size_t npix = (size_t)in->W * in->H;
  if (!r->ws && npix > r->capPix) {  // a workspace forward is forward-only: no per-pixel state
    int rc;
    if ((rc = grow((void**)&r->final_T, npix * sizeof(float)))) return rc;
    if ((rc = grow((void**)&r->n_contrib, npix * sizeof(int)))) return rc;
    r->capPix = npix;
  }
  // GSMPM_RASTER_WIDE_KEYS=1 forces upstream's 64-bit (tile, depth) keys (tests compare the two)
  const char* wide = std::getenv("GSMPM_RASTER_WIDE_KEYS");
  const bool depth_ordered = !(wide && wide[0] == '1');
  // GSMPM_RASTER_RENDER_MODE=1 disables k_render's sub-tile culling (tests
  // check that culling changes no pixel, final T or last contributor)
  const char* rm = std::getenv("GSMPM_RASTER_RENDER_MODE");
  const int render_mode = rm ? std::atoi(rm) & 1 : 0;
  a.tight = !(render_mode & 1);
  // the chunked tile sort (<= kMaxTiles tiles; GSMPM_RASTER_ONESWEEP=1 forces rocPRIM onesweep everywhere)
  const char* os = std::getenv("GSMPM_RASTER_ONESWEEP");
  const bool force_onesweep = os && os[0] == '1';
  // GSMPM_RASTER_CHUNKED=0: the LSD digit sort below kMaxTiles tiles too (A/B)
  const char* ck = std::getenv("GSMPM_RASTER_CHUNKED");
  const bool chunked = ntiles <= (size_t)kMaxTiles && !force_onesweep && !(ck && ck[0] == '0');
  // GSMPM_RASTER_TILE_DSORT=1 (chunked path): depth order per tile after the tile sort (k_tile_dsort)
  // instead of the global depth sort before the emission.  Bit-identical (the raster, golden, e2e and
  // config tests pass with it) but slower: lego render alone 0.311 vs 0.194 ms (3 rounds), so off
  const char* td = std::getenv("GSMPM_RASTER_TILE_DSORT");
  const bool tile_dsort = depth_ordered && chunked && td && td[0] == '1';
  a.sh_vec4 = in->shs && in->M == 16 && ((uintptr_t)in->shs & 15u) == 0;
  r->slots_pending = false;
  r->offsets_pending = false;
  r->emit_culled = false;
  const unsigned* tkeys = nullptr;  // sorted tile keys with sub-tile masks (chunked path)
  const unsigned* async_over = nullptr;  // the async form's bucket-overflow flag (device state, bucket form)
  unsigned K = 0, K_full = 0;  // binned pairs, upstream's 3-sigma pairs (num_rendered)
  if (P > 0) {
    // GSMPM_RASTER_DSORT=lib: the library's radix sort + scan for the depth order (A/B; also the
    // fallback when a depth bucket overflows, dsort.h)
    // GSMPM_RASTER_DSORT=bucket / lsd force a form of the hand-written one
    // (default: the LSD form from kDlMin Gaussians, the bucket form below)
    const char* dl = std::getenv("GSMPM_RASTER_DSORT");
    const bool lib_dsort = dl && std::strcmp(dl, "lib") == 0;
    const bool own_dsort = depth_ordered && !tile_dsort && !lib_dsort;
    const bool lsd_dsort = own_dsort && (dl && std::strcmp(dl, "lsd") == 0 ? true
                                         : dl && std::strcmp(dl, "bucket") == 0 ? false
                                                                                : P >= kDlMin);
    const DsortBufs db = dsort_bufs(r);
    hipLaunchKernelGGL(k_preprocess, dim3(div_up(P, 256)), dim3(256), 0, st, a, out_radii, r->depth, r->xy, r->conic,
                       r->rgb, r->tiles, r->rect, own_dsort ? db.shard : nullptr);
    GSMPM_LAUNCH_CHECK();
    // the index-order scan (offsets) feeds only the backward's record slots
    // and the upstream-keyed path: a depth-ordered forward takes K from the
    // depth-order scan and leaves offsets to gsmpm_raster_backward (one scan
    // and its look-back init launch less per frame)
    r->offsets_pending = true;
    if (!depth_ordered || tile_dsort)  // the index-order scan of both counts (emission offsets, K)
      scan_tiles<unsigned long long>(r, P, r->offr, st);
    auto lib_depth_order = [&]() -> int {
      size_t b2 = r->dsort_tmp_bytes;
      if (kDepthOnesweepMin > 0 && (size_t)P >= kDepthOnesweepMin)
        GSMPM_HIP(rocprim::radix_sort_pairs<OnesweepSort>(r->dsort_tmp, b2, reinterpret_cast<unsigned*>(r->depth),
                                                          r->dsorted, rocprim::counting_iterator<unsigned>(0u),
                                                          r->dorder, (size_t)P, 0, 32, st));
      else
        GSMPM_HIP(rocprim::radix_sort_pairs(r->dsort_tmp, b2, reinterpret_cast<unsigned*>(r->depth), r->dsorted,
                                            rocprim::counting_iterator<unsigned>(0u), r->dorder, (size_t)P, 0, 32,
                                            st));
      // the scan reads tiles[dorder[r]] itself (no separate gather launch)
      b2 = r->scan_tmp_bytes;
      GSMPM_HIP(rocprim::inclusive_scan(r->scan_tmp, b2, ranked_tiles(r->dorder, r->tiles), r->offr, (size_t)P,
                                        rocprim::plus<unsigned long long>(), st));
      return GSMPM_OK;
    };
    // K straight into pinned, coherent host memory by the depth order's own
    // last kernels (dsort.h ds_publish; the library path: a one-lane kernel),
    // and a spin on it: no copy-engine packet and no sleeping stream sync
    // between the scan and the post-count launches.  Every 256 polls the event
    // recorded behind the publishing kernels is queried, so a device fault
    // surfaces at once instead of after a timeout; a completed event with no
    // count is an error.  The count needs the host, so a capturing stream is
    // refused.
    const bool async = r->async_cap > 0;  // the pair count stays on the device (gsmpm_raster_forward_async)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    GSMPM_HIP(hipStreamIsCapturing(st, &cap));
    GSMPM_REQUIRE(async || cap == hipStreamCaptureStatusNone,
                  "gsmpm_raster_forward: the pair count is read on the host; the stream must not be capturing");
    volatile unsigned* hc = r->h_count;
    auto arm = [&]() {
      hc[0] = kNoCount;
      hc[1] = kNoCount;
      hc[2] = 0;
      hc[3] = 1;
    };
    auto wait_count = [&]() -> int {
      GSMPM_HIP(hipEventRecord(r->count_ev, st));
      for (unsigned polls = 1; *hc == kNoCount; ++polls) {
        if ((polls & 255) == 0) {
          const hipError_t q = hipEventQuery(r->count_ev);
          if (q == hipSuccess) break;  // everything up to the publish finished: K is visible below
          if (q != hipErrorNotReady) GSMPM_HIP(q);
        }
        __builtin_ia32_pause();
      }
      return GSMPM_OK;
    };
    auto publish = [&](const unsigned* over) -> int {  // a one-lane kernel behind everything so far
      arm();
      hipLaunchKernelGGL(k_publish_count, dim3(1), dim3(1), 0, st, (const unsigned long long*)(r->offr + (P - 1)),
                         over, r->h_count);
      GSMPM_LAUNCH_CHECK();
      return wait_count();
    };
    // GSMPM_RASTER_EARLY_COUNT=0: the hand-written depth order leaves the publish to the one-lane
    // kernel after its last launch, as rounds 1-3 did (A/B)
    const char* ec = std::getenv("GSMPM_RASTER_EARLY_COUNT");
    const bool early = own_dsort && !(ec && ec[0] == '0');
    unsigned* pub = async ? r->async_counts : early ? r->h_count : nullptr;
    // the depth order depends on P only: it runs before the count read-back,
    // queued behind whatever the stream is still doing
    if (early && !async) arm();  // before the kernels that publish
    // the LSD form; from_state = 1: the bucket form's overflow fallback (lo from its state, all 4 passes)
    auto lsd_depth_order = [&](int from_state, unsigned* pubp) {
      const DlBufs b = dl_bufs(r, P);
      const int nch = div_up(P, kDlChunk);
      const float* dp = r->depth;
      const unsigned long long* tw = r->tiles;
      // digit rows of >= 128 chunks (>= 262,144 Gaussians): a workgroup per row
      auto rows = [&](int pass) {
        if (nch >= 128 && nch <= kRowsWideMax)
          hipLaunchKernelGGL(k_rows_wide, dim3(256), dim3(256), nch * sizeof(unsigned), st, nch, (const unsigned*)b.H,
                             b.Hs, b.tot, pass ? (const unsigned*)(b.st + DS_DL_NB1) : nullptr, 8u * pass);
        else
          hipLaunchKernelGGL(k_dl_rows, dim3(64), dim3(256), 0, st, nch, pass, b);
      };
      for (int pass = 0; pass < kDlPasses; ++pass) {
        if (pass == 0) {
          hipLaunchKernelGGL(k_dl_hist<true>, dim3(nch), dim3(256), 0, st, P, nch, pass, dp, tw, b, from_state);
          rows(pass);
          hipLaunchKernelGGL(k_dl_scatter<true>, dim3(nch), dim3(256), 0, st, P, nch, pass, dp, tw, b, from_state);
        } else {
          hipLaunchKernelGGL(k_dl_hist<false>, dim3(nch), dim3(256), 0, st, P, nch, pass, dp, tw, b, from_state);
          rows(pass);
          hipLaunchKernelGGL(k_dl_scatter<false>, dim3(nch), dim3(256), 0, st, P, nch, pass, dp, tw, b, from_state);
        }
      }
      const int nsb = div_up(P, kScanBlk);
      hipLaunchKernelGGL(k_dl_scan_blocks, dim3(nsb), dim3(256), 0, st, P, tw, b, r->scan_bt);
      hipLaunchKernelGGL(k_dl_scan_apply, dim3(nsb), dim3(256), 0, st, P, tw, b,
                         (const unsigned long long*)r->scan_bt, r->dorder, r->offr, pubp);
    };
    if (lsd_dsort) {
      lsd_depth_order(0, pub);
      GSMPM_LAUNCH_CHECK();
    } else if (own_dsort) {
      const int nb = dsort_buckets(P);
      hipLaunchKernelGGL(k_dsort_hist, dim3(div_up(P, 256)), dim3(256), 0, st, P, nb, (const float*)r->depth,
                         (const unsigned long long*)r->tiles, db);
      hipLaunchKernelGGL(k_dsort_scan1, dim3(nb / kDsBlk), dim3(256), 0, st, db, db.btc, db.bts);
      hipLaunchKernelGGL(k_dsort_scan2, dim3(nb / kDsBlk), dim3(256), 0, st, nb, db, (const unsigned*)db.btc,
                         (const unsigned long long*)db.bts, pub);
      hipLaunchKernelGGL(k_dsort_scatter, dim3(div_up(P, 256)), dim3(256), 0, st, P, (const float*)r->depth,
                         (const unsigned long long*)r->tiles, db, r->dorder, r->offr);
      // a wave per bucket, up to one bucket per wave at ~8 Gaussians a bucket (one pass: the loop's
      // dependent loads -- list entry, bucket record, keys -- are the cost)
      hipLaunchKernelGGL(k_dsort_small, dim3((unsigned)std::max(1, std::min(16384, div_up(std::min(nb, P), 4)))),
                         dim3(256), 0, st, (const unsigned long long*)r->tiles, db, r->dorder, r->offr);
      // the buckets above kDsSmall: launched after the count when it says there are any (early
      // publish), else here, before the one-lane publish reads the last element
      if (!early)
        hipLaunchKernelGGL(k_dsort_big, dim3(256), dim3(1024), 0, st, (const unsigned long long*)r->tiles, db,
                           r->dorder, r->offr);
      GSMPM_LAUNCH_CHECK();
    } else if (depth_ordered && !tile_dsort) {
      const int rc = lib_depth_order();
      if (rc) return rc;
    }
    if (async) {
      // no host read: the buckets above kDsSmall always get k_dsort_big (it exits
      // at once without any), an overflowing bucket is the caller's flag (counts[2]:
      // the frame is rendered again by the synchronous form), and the pair
      // buffers hold async_cap pairs (counts[2] bit 1 when the frame needs more)
      if (!lsd_dsort) {
        hipLaunchKernelGGL(k_dsort_big, dim3(256), dim3(1024), 0, st, (const unsigned long long*)r->tiles, db,
                           r->dorder, r->offr);
        GSMPM_LAUNCH_CHECK();
      }
      K = (unsigned)r->async_cap;
      K_full = 0;
      if (!lsd_dsort) async_over = db.st + DS_OVERD;
    }
    int rc = async ? GSMPM_OK : early ? wait_count() : publish(own_dsort && !lsd_dsort ? db.st + DS_OVERD : nullptr);
    if (rc) return rc;
    if (!async && early && !lsd_dsort && hc[3]) {
      hipLaunchKernelGGL(k_dsort_big, dim3(256), dim3(1024), 0, st, (const unsigned long long*)r->tiles, db,
                         r->dorder, r->offr);
      GSMPM_LAUNCH_CHECK();
    }
    if (!async && own_dsort && !lsd_dsort && hc[2]) {
      // a depth bucket above kDsBig entries (a degenerate depth distribution): the
      // hand-written LSD form from the bucket form's state instead (dsort.h)
      r->dsort_fallbacks += 1;
      arm();
      lsd_depth_order(1, r->h_count);
      GSMPM_LAUNCH_CHECK();
      if ((rc = wait_count())) return rc;
    }
    if (!async) {
      K = hc[0];
      K_full = hc[1];
      GSMPM_REQUIRE(K != kNoCount && K_full != kNoCount, "gsmpm_raster_forward: the pair count never arrived");
    }
  }
  if (K > 0 && r->ws) {
    const int rc = ws_carve_pairs(r, K, ntiles);
    if (rc) return rc;
  }
  if (K > 0) {
    if (K > r->capK) {
      const size_t cap = (size_t)K + K / 4 + 1024;
      int rc;
      if ((rc = grow((void**)&r->keys, cap * 8))) return rc;
      if ((rc = grow((void**)&r->keys_sorted, cap * 8))) return rc;
      if ((rc = grow((void**)&r->vals, cap * 4))) return rc;
      if ((rc = grow((void**)&r->vals_sorted, cap * 4))) return rc;
      if ((rc = grow((void**)&r->ids_sorted, cap * 4))) return rc;
      if ((rc = grow((void**)&r->estart, (cap / kEmitT + 2) * 4))) return rc;
      size_t bytes = 0;
      GSMPM_HIP(rocprim::radix_sort_pairs(nullptr, bytes, r->keys, r->keys_sorted, rocprim::counting_iterator<unsigned>(0u),
                                          r->vals_sorted, cap, 0, 64, st));
      if ((rc = grow(&r->sort_tmp, bytes))) return rc;
      r->sort_tmp_bytes = bytes;
      r->capK = cap;
    }
    const int bits = msb_bits((unsigned)ntiles);
    // the async form: the kernels cut at the device's count (offr's last entry)
    const unsigned long long* kdev = r->async_cap > 0 ? (const unsigned long long*)(r->offr + (P - 1)) : nullptr;
    if (depth_ordered) {
      unsigned* tile_keys = reinterpret_cast<unsigned*>(r->keys);
      unsigned* tile_sorted = reinterpret_cast<unsigned*>(r->keys_sorted);
      // the chunked counting sort needs the tile histogram in LDS; above kMaxTiles
      // tiles the LSD digit sort (k_lsd_*).  GSMPM_RASTER_LSD=0: the library's
      // onesweep above kMaxTiles instead; GSMPM_RASTER_ONESWEEP=1 forces it everywhere
      const char* ls = std::getenv("GSMPM_RASTER_LSD");
      const bool digits = !chunked && !force_onesweep && !(ls && ls[0] == '0');
      const int passes = (bits + 7) / 8;  // ntiles <= 256^passes - 1: the all-ones tile field stays the culled one
      const int nch = (int)div_up(K, kChunk);
      // 8,192-pair chunks for the digit sort (lsd.h): bicycle render 1.078-1.080 against
      // 1.082-1.088 ms with 4,096 (3 rounds, profiles/r04/render/ab_lsd_chunk_r04i.txt);
      // GSMPM_RASTER_LSD_I=16 restores 4,096 (A/B)
      const char* li = std::getenv("GSMPM_RASTER_LSD_I");
      const bool lsd32 = !(li && std::atoi(li) == 16);
      const int nchl = (int)div_up(K, lsd32 ? 32 * kLsdT : kLsdChunk);
      // digit rows of at least this many chunks: a workgroup per row (k_rows_wide); tests lower it
      const char* rw = std::getenv("GSMPM_RASTER_ROWS_WIDE_MIN");
      const int rows_wide_min = rw ? std::atoi(rw) : kRowsWideMin;
      size_t need = 0;
      if (digits) {
        const size_t nh = 256 * (size_t)nchl;
        if (nh > r->capH) {
          int rc;
          if ((rc = grow((void**)&r->hist, 2 * (nh + nh / 4 + 1024) * sizeof(unsigned)))) return rc;
          r->capH = nh + nh / 4 + 1024;
        }
      } else if (chunked) {
        const size_t nh = (ntiles + 1) * (size_t)nch;
        if (nh > r->capH) {
          int rc;
          if ((rc = grow((void**)&r->hist, 2 * (nh + nh / 4 + 1024) * sizeof(unsigned)))) return rc;
          r->capH = nh + nh / 4 + 1024;
        }
      } else {
        GSMPM_HIP(rocprim::radix_sort_pairs<OnesweepSort>(nullptr, need, tile_keys, tile_sorted, r->vals,
                                                          r->ids_sorted, (size_t)K, 0, bits, st));
      }
      if (need > r->sort_tmp_bytes) {
        int rc;
        if ((rc = grow(&r->sort_tmp, need))) return rc;
        r->sort_tmp_bytes = need;
      }
      // sub-tile masks in the keys' top bits (every sort orders the tile bits only)
      const int cull = !(render_mode & 1);
      const char* el = std::getenv("GSMPM_RASTER_EMIT_LANE");
      if (el && el[0] == '1') {
        hipLaunchKernelGGL(k_emit_pairs, dim3(div_up(K, 256)), dim3(256), 0, st, (int)K, P,
                           tile_dsort ? nullptr : (const unsigned*)r->dorder,
                           (const unsigned long long*)r->offr, (const float2*)r->xy, (const float4*)r->conic,
                           (const uint2*)r->rect, a.grid_x, cull, tile_keys, r->vals);
      } else {  // >= ~1024 workgroups, up to kEmitMaxI pairs per lane
        const int items = std::min(kEmitMaxI, std::max(1, div_up((long)K, (long)kEmitT * 1024)));
        const int nwg = div_up((long)K, (long)kEmitT * items);
        hipLaunchKernelGGL(k_emit_starts, dim3(div_up(P, 256)), dim3(256), 0, st, P, (const unsigned long long*)r->offr,
                           (unsigned)(kEmitT * items), r->estart, (unsigned)(nwg + 1), K, async_over,
                           r->async_cap > 0 ? r->async_counts + 2 : nullptr);
        GSMPM_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_emit_wg, dim3(nwg), dim3(kEmitT), 0, st, (int)K, P, items, (const unsigned*)r->estart,
                           tile_dsort ? nullptr : (const unsigned*)r->dorder, (const unsigned long long*)r->offr,
                           (const float2*)r->xy,
                           (const float4*)r->conic, (const uint2*)r->rect, a.grid_x, cull, tile_keys, r->vals, kdev);
      }
      GSMPM_LAUNCH_CHECK();
      size_t bytes = r->sort_tmp_bytes;
      if (chunked) {
        unsigned* Hs = r->hist + r->capH;
        hipLaunchKernelGGL(k_tile_hist, dim3(nch), dim3(kSortT), 0, st, (int)K, (int)ntiles, nch, bits,
                           (const unsigned*)tile_keys, r->hist, kdev);
        GSMPM_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_tile_rows, dim3(div_up((long)ntiles + 1, 4)), dim3(256), 0, st, (int)ntiles, nch,
                           (const unsigned*)r->hist, Hs, r->ttot);
        hipLaunchKernelGGL(k_tile_scatter, dim3(nch), dim3(kSortT), 0, st, (int)K, (int)ntiles, nch, bits,
                           (const unsigned*)tile_keys, (const unsigned*)r->vals, (const unsigned*)Hs,
                           (const unsigned*)r->ttot, tile_sorted,
                           r->ids_sorted, r->ranges, tile_dsort ? r->dsort_tl : nullptr, kdev);
        GSMPM_LAUNCH_CHECK();
        if (tile_dsort) {  // depth order within each tile's list (the emission keys are dead: scratch)
          hipLaunchKernelGGL((k_tile_dsort<kDsortSmall, false>), dim3((unsigned)ntiles), dim3(256), 0, st,
                             (const uint2*)r->ranges, (int)ntiles, (const float*)r->depth, tile_sorted, r->ids_sorted,
                             r->dsort_tl);
          hipLaunchKernelGGL((k_tile_dsort<kDsortLarge, true>), dim3(256), dim3(256), 0, st, (const uint2*)r->ranges,
                             (int)ntiles, (const float*)r->depth, tile_sorted, r->ids_sorted, r->dsort_tl);
          hipLaunchKernelGGL(k_tile_dsort_rank, dim3(64), dim3(256), 0, st, (const uint2*)r->ranges, (int)ntiles,
                             (const float*)r->depth, tile_sorted, r->ids_sorted, (const int*)r->dsort_tl,
                             tile_keys, tile_keys + r->capK);
          GSMPM_LAUNCH_CHECK();
        }
        tkeys = tile_sorted;
        r->emit_culled = cull != 0;
        ranges_written = true;
      } else {
        if (digits) {  // passes alternate between the final buffers and spare ones, ending in the final
          unsigned* Hs = r->hist + r->capH;
          unsigned* alt_k = tile_keys + r->capK;  // the upper half of the 8-byte key buffer
          unsigned* alt_v = r->vals_sorted;       // (the backward's slots; free in the forward)
          const unsigned *sk = tile_keys, *sv = r->vals;
          for (int p = 0; p < passes; ++p) {
            const bool fin = (passes - 1 - p) % 2 == 0;
            unsigned* dk = fin ? tile_sorted : alt_k;
            unsigned* dv = fin ? r->ids_sorted : alt_v;
            if (lsd32)
              hipLaunchKernelGGL(k_lsd_hist<32>, dim3(nchl), dim3(kLsdT), 0, st, (int)K, nchl, 8 * p, sk, r->hist);
            else
              hipLaunchKernelGGL(k_lsd_hist<kLsdI>, dim3(nchl), dim3(kLsdT), 0, st, (int)K, nchl, 8 * p, sk, r->hist);
            if (nchl >= rows_wide_min && nchl <= kRowsWideMax)
              hipLaunchKernelGGL(k_rows_wide, dim3(256), dim3(256), nchl * sizeof(unsigned), st, nchl,
                                 (const unsigned*)r->hist, Hs, r->ttot, (const unsigned*)nullptr, 0u);
            else
              hipLaunchKernelGGL(k_tile_rows, dim3(64), dim3(256), 0, st, 255, nchl, (const unsigned*)r->hist, Hs,
                                 r->ttot);
            if (lsd32)
              hipLaunchKernelGGL(k_lsd_scatter<32>, dim3(nchl), dim3(kLsdT), 0, st, (int)K, nchl, 8 * p, sk, sv,
                                 (const unsigned*)Hs, (const unsigned*)r->ttot, dk, dv);
            else
              hipLaunchKernelGGL(k_lsd_scatter<kLsdI>, dim3(nchl), dim3(kLsdT), 0, st, (int)K, nchl, 8 * p, sk, sv,
                                 (const unsigned*)Hs, (const unsigned*)r->ttot, dk, dv);
            GSMPM_LAUNCH_CHECK();
            sk = dk;
            sv = dv;
          }
        } else {
          GSMPM_HIP(rocprim::radix_sort_pairs<OnesweepSort>(r->sort_tmp, bytes, tile_keys, tile_sorted, r->vals,
                                                            r->ids_sorted, (size_t)K, 0, bits, st));
        }
        GSMPM_HIP(hipMemsetAsync(r->ranges, 0, ntiles * sizeof(uint2), st));
        hipLaunchKernelGGL(k_ranges32, dim3(div_up(K, 1024)), dim3(256), 0, st, (int)K, (const unsigned*)tile_sorted,
                           (unsigned)ntiles, r->ranges);
        GSMPM_LAUNCH_CHECK();
        tkeys = tile_sorted;
        r->emit_culled = cull != 0;
      }
      r->slots_pending = true;
    } else {
    hipLaunchKernelGGL(k_duplicate, dim3(div_up(P, 256)), dim3(256), 0, st, P, (const uint2*)r->rect, r->depth,
                       (const unsigned long long*)r->offr, out_radii, a.grid_x, r->keys, r->vals);
    GSMPM_LAUNCH_CHECK();
    size_t bytes = r->sort_tmp_bytes;
    // values = emission indices (a Gaussian's pairs are contiguous in emission order: the
    // backward sums them without atomics); ids_sorted maps them back to Gaussians
    GSMPM_HIP(rocprim::radix_sort_pairs(r->sort_tmp, bytes, r->keys, r->keys_sorted,
                                        rocprim::counting_iterator<unsigned>(0u), r->vals_sorted, (size_t)K, 0,
                                        32 + bits, st));
    hipLaunchKernelGGL(k_ids, dim3(div_up(K, 256)), dim3(256), 0, st, (int)K, r->vals_sorted, r->vals, r->ids_sorted);
    GSMPM_HIP(hipMemsetAsync(r->ranges, 0, ntiles * sizeof(uint2), st));
    hipLaunchKernelGGL(k_ranges, dim3(div_up(K, 256)), dim3(256), 0, st, (int)K, r->keys_sorted, r->ranges);
    GSMPM_LAUNCH_CHECK();
    }
  }
  if (!ranges_written && K == 0) GSMPM_HIP(hipMemsetAsync(r->ranges, 0, ntiles * sizeof(uint2), st));
  // GSMPM_RASTER_TILE_SHARED=1: k_render4 (one workgroup per tile; bit-identical output).  It
  // moves 35 % fewer bytes (lego frame: 41.3 vs 63.6 MB per launch, PMC) but renders in
  // 0.30-0.33 ms against 0.26-0.27 ms (tools/ab_render.sh, 3 pairs): the blend is bound by
  // the heaviest tiles' serial walk, and a tile's four quarters now wait for each other
  const char* ts = std::getenv("GSMPM_RASTER_TILE_SHARED");
  // GSMPM_RASTER_XCD=0: the row-major 2-D grid of quarters instead of the XCD-grouped one
  const char* xe = std::getenv("GSMPM_RASTER_XCD");
  const int xcd = !(xe && xe[0] == '0');
  const int nq = xcd ? (int)(32 * div_up((long)ntiles, 8)) : 2 * a.grid_x;  // the 2-D grid: one pass per workgroup
  dim3 rgrid = xcd ? dim3((unsigned)nq) : dim3(2 * a.grid_x, 2 * a.grid_y);
  // GSMPM_RASTER_RENDER_WGS=N (a multiple of 8): k_render as N workgroups looping over the quarters
  // (A/B: a render overlapping the simulator holds fewer of the CU slots its one-round launches need)
  if (const char* rw = std::getenv("GSMPM_RASTER_RENDER_WGS"))
    if (xcd && std::atoi(rw) >= 8) rgrid = dim3((unsigned)std::min(nq, std::atoi(rw) & ~7));
  tmg.mark(1);
  if (!(ts && ts[0] == '1'))
    hipLaunchKernelGGL(k_render, rgrid, dim3(64), 0, st, r->ranges, r->ids_sorted, a.W, a.H, a.grid_x, r->xy, r->conic,
                       r->rgb, in->bg, out_color, r->forward_only ? nullptr : r->final_T,
                       r->forward_only ? nullptr : r->n_contrib, tkeys, render_mode, xcd, (int)ntiles, nq);
  else
    hipLaunchKernelGGL(k_render4, dim3(a.grid_x, a.grid_y), dim3(256), 0, st, r->ranges, r->ids_sorted, a.W, a.H,
                       a.grid_x, r->xy, r->conic, r->rgb, in->bg, out_color, r->forward_only ? nullptr : r->final_T,
                       r->forward_only ? nullptr : r->n_contrib, tkeys, render_mode);
  tmg.mark(2);
  r->has_pixel_state = !r->forward_only;
  GSMPM_LAUNCH_CHECK();
  if (num_rendered) *num_rendered = r->async_cap > 0 ? -1 : (int32_t)K_full;
  r->P = P;
  r->W = a.W;
  r->H = a.H;
  r->gx = a.grid_x;
  r->gy = a.grid_y;
  r->K = K;
  r->K_full = K_full;
  return GSMPM_OK;
}

int gsmpm_raster_backward(gsmpm_raster* r, const gsmpm_raster_args* in, const int32_t* radii, const float* dL_dcolor,
                          float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                          float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations, void* stream) {
  GSMPM_REQUIRE(r && in && radii && dL_dcolor && dL_dmeans2D && dL_dcolors && dL_dopacity && dL_dmeans3D && dL_dcov3D,
                "gsmpm_raster_backward: null argument");
  GSMPM_REQUIRE(r->P == in->P && r->W == in->W && r->H == in->H,
                "gsmpm_raster_backward: the context holds no forward of these sizes (one context per differentiable forward)");
  GSMPM_REQUIRE(r->has_pixel_state || in->P == 0,
                "gsmpm_raster_backward: the context's forward was forward-only (gsmpm_raster_set_forward_only)");
  GSMPM_REQUIRE(!in->shs || dL_dsh, "gsmpm_raster_backward: shs given but no dL_dsh output");
  GSMPM_REQUIRE(!in->scales || (dL_dscales && dL_drotations), "gsmpm_raster_backward: scales given but no outputs");
  hipStream_t st = (hipStream_t)stream;
  if (in->P == 0) return GSMPM_OK;
  RasterDev a;
  a.P = in->P; a.D = in->D; a.M = in->M; a.W = in->W; a.H = in->H;
  a.means3D = in->means3D; a.shs = in->shs; a.colors_precomp = in->colors_precomp; a.opacities = in->opacities;
  a.scales = in->scales; a.rotations = in->rotations; a.cov3D_precomp = in->cov3D_precomp;
  a.scale_modifier = in->scale_modifier; a.viewmatrix = in->viewmatrix; a.projmatrix = in->projmatrix;
  a.campos = in->campos; a.bg = in->bg; a.tanfovx = in->tanfovx; a.tanfovy = in->tanfovy;
  a.focal_x = in->W / (2.0f * in->tanfovx);
  a.focal_y = in->H / (2.0f * in->tanfovy);
  a.grid_x = r->gx; a.grid_y = r->gy;
  a.tight = 0; a.sh_vec4 = 0;  // forward-only fields
  const size_t K = r->K;
  if (K > r->capRec) {
    int rc;
    if ((rc = grow((void**)&r->rec, (K + K / 4 + 1024) * 3 * sizeof(float4)))) return rc;
    r->capRec = K + K / 4 + 1024;
  }
  if (r->offsets_pending) {  // the forward's tiles are still in r->tiles
    scan_tiles<unsigned>(r, in->P, r->offsets, st);
    GSMPM_LAUNCH_CHECK();
    r->offsets_pending = false;
  }
  if (K > 0 && r->slots_pending) {
    hipLaunchKernelGGL(k_slots, dim3(div_up(K, 256)), dim3(256), 0, st, (int)K,
                       (const unsigned*)reinterpret_cast<unsigned*>(r->keys_sorted), (const unsigned*)r->ids_sorted,
                       (const uint2*)r->rect, (const unsigned*)r->offsets, r->gx, r->gy, r->vals_sorted);
    GSMPM_LAUNCH_CHECK();
    r->slots_pending = false;
  }
  if (K > 0 && r->emit_culled) GSMPM_HIP(hipMemsetAsync(r->rec, 0, K * 3 * sizeof(float4), st));
  const char* poison = std::getenv("GSMPM_RASTER_POISON");
  if (K > 0 && poison && poison[0] == '1') {
    hipLaunchKernelGGL(k_poison_listed, dim3(r->gx * r->gy), dim3(256), 0, st, (const uint2*)r->ranges,
                       (const unsigned*)r->vals_sorted, r->rec);
    GSMPM_LAUNCH_CHECK();
  }
  if (K > 0)
    hipLaunchKernelGGL(k_render_bwd, dim3(r->gx, r->gy), dim3(kBlock), 0, st, r->ranges, r->vals_sorted,
                       r->ids_sorted, a.W, a.H, r->gx, r->xy, r->conic, r->rgb, in->bg, r->final_T, r->n_contrib,
                       dL_dcolor, r->rec);
  RasterGrads o{dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations};
  hipLaunchKernelGGL(k_preprocess_bwd, dim3(div_up(a.P, 256)), dim3(256), 0, st, a, radii, r->offsets, r->rgb,
                     r->rec, o);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

int gsmpm_raster_pair_counts(const gsmpm_raster* r, uint32_t* binned, uint32_t* rendered) {
  GSMPM_REQUIRE(r, "gsmpm_raster_pair_counts: null context");
  if (binned) *binned = r->K;
  if (rendered) *rendered = r->K_full;
  return GSMPM_OK;
}

int gsmpm_raster_set_forward_only(gsmpm_raster* r, int32_t on) {
  GSMPM_REQUIRE(r, "gsmpm_raster_set_forward_only: null context");
  r->forward_only = on != 0;
  return GSMPM_OK;
}

int gsmpm_raster_dsort_stats(const gsmpm_raster* r, int64_t out8[8]) {
  GSMPM_REQUIRE(r && out8, "gsmpm_raster_dsort_stats: null argument");
  unsigned st[kDsWords] = {0};
  if (r->ds_state) GSMPM_HIP(hipMemcpy(st, r->ds_state, sizeof(st), hipMemcpyDeviceToHost));
  out8[0] = st[DS_NB];
  out8[1] = st[DS_NLIST];
  out8[2] = st[DS_NBIG];
  out8[3] = st[DS_MAXN];
  out8[4] = st[DS_OVERD];
  out8[5] = st[DS_PV];
  out8[6] = r->dsort_fallbacks;
  out8[7] = st[DS_SHIFT];
  return GSMPM_OK;
}

int gsmpm_raster_workspace_size(int32_t P, int32_t H, int32_t W, int64_t pairs, uint64_t* bytes) {
  GSMPM_REQUIRE(bytes && P >= 0 && H > 0 && W > 0 && pairs >= 0, "gsmpm_raster_workspace_size: bad argument");
  const size_t ntiles = (size_t)div_up(W, kBX) * (size_t)div_up(H, kBY);
  gsmpm_raster tmp;
  WsWalk w{nullptr, 0};
  int rc = ws_pre_walk(w, &tmp, (size_t)P, ntiles);
  if (!rc) rc = ws_pairs_walk(w, &tmp, (size_t)pairs, ntiles);
  if (rc) return rc;
  *bytes = (uint64_t)w.off;
  return GSMPM_OK;
}

// the pinned pair-count word and its event for workspace forwards: one per
// thread and device (a workspace forward holds no context)
struct WsCount {
  unsigned* h = nullptr;
  hipEvent_t ev = nullptr;
};
static int ws_count(WsCount*& out) {
  static thread_local std::vector<WsCount> per_dev;
  int dev = 0;
  GSMPM_HIP(hipGetDevice(&dev));
  if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1);
  WsCount& c = per_dev[dev];
  if (!c.h) {
    GSMPM_HIP(hipHostMalloc((void**)&c.h, 4 * sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    GSMPM_HIP(hipEventCreateWithFlags(&c.ev, hipEventDisableTiming));
  }
  out = &c;
  return GSMPM_OK;
}

int gsmpm_raster_forward_ws(const gsmpm_raster_args* a, float* out_color, int32_t* out_radii, int32_t* num_rendered,
                            void* workspace, uint64_t ws_bytes, int64_t* pairs_needed, void* stream) {
  GSMPM_REQUIRE(a && workspace && ((uintptr_t)workspace & 255u) == 0,
                "gsmpm_raster_forward_ws: null argument or workspace not 256-byte aligned");
  GSMPM_REQUIRE(a->P >= 0 && a->W > 0 && a->H > 0, "gsmpm_raster_forward_ws: bad sizes");
  if (pairs_needed) *pairs_needed = 0;
  WsCount* c = nullptr;
  int rc = ws_count(c);
  if (rc) return rc;
  gsmpm_raster r;  // a view of the workspace: nothing in it is allocated or freed
  r.forward_only = true;
  r.h_count = c->h;
  r.count_ev = c->ev;
  r.ws = reinterpret_cast<char*>(workspace);
  r.ws_bytes = (size_t)ws_bytes;
  const size_t ntiles = (size_t)div_up(a->W, kBX) * (size_t)div_up(a->H, kBY);
  WsWalk w{r.ws, 0};
  rc = ws_pre_walk(w, &r, (size_t)a->P, ntiles);
  if (rc) return rc;
  r.ws_pre = w.off;
  if (r.ws_pre > r.ws_bytes) {
    if (pairs_needed) *pairs_needed = 0;
    set_error("gsmpm_raster_forward_ws: the workspace is smaller than gsmpm_raster_workspace_size(P, H, W, 0)");
    return GSMPM_ESPACE;
  }
  rc = gsmpm_raster_forward(&r, a, out_color, out_radii, num_rendered, stream);
  if (rc == GSMPM_ESPACE && pairs_needed) *pairs_needed = r.pairs_needed;
  return rc;
}

int gsmpm_raster_forward_async(const gsmpm_raster_args* a, float* out_color, int32_t* out_radii, void* workspace,
                               uint64_t ws_bytes, int64_t pairs_cap, uint32_t* counts, void* stream) {
  GSMPM_REQUIRE(a && out_color && (out_radii || a->P == 0) && counts && workspace && ((uintptr_t)workspace & 255u) == 0,
                "gsmpm_raster_forward_async: null argument or workspace not 256-byte aligned");
  GSMPM_REQUIRE(a->P >= 0 && a->W > 0 && a->H > 0 && pairs_cap > 0 && pairs_cap < (1LL << 31),
                "gsmpm_raster_forward_async: bad sizes or pairs_cap");
  const size_t ntiles = (size_t)div_up(a->W, kBX) * (size_t)div_up(a->H, kBY);
  // the paths whose launch sizes do not depend on the pair count: the default
  // depth-ordered forward with the chunked tile sort (<= kMaxTiles tiles)
  auto env_is = [](const char* k, const char* v) {
    const char* e = std::getenv(k);
    return e && std::strcmp(e, v) == 0;
  };
  GSMPM_REQUIRE(ntiles <= (size_t)kMaxTiles, "gsmpm_raster_forward_async: more than 4,096 tiles (the digit sort "
                "sizes its passes by the pair count): use gsmpm_raster_forward_ws");
  GSMPM_REQUIRE(!env_is("GSMPM_RASTER_WIDE_KEYS", "1") && !env_is("GSMPM_RASTER_ONESWEEP", "1") &&
                    !env_is("GSMPM_RASTER_CHUNKED", "0") && !env_is("GSMPM_RASTER_TILE_DSORT", "1") &&
                    !env_is("GSMPM_RASTER_DSORT", "lib") && !env_is("GSMPM_RASTER_EMIT_LANE", "1"),
                "gsmpm_raster_forward_async: an A/B switch selects a path the async form does not take");
  hipStream_t st = (hipStream_t)stream;
  if (a->P == 0) {  // the image is the background; every count is 0
    hipLaunchKernelGGL(k_fill_bg, dim3(div_up((long)a->W * a->H, 256)), dim3(256), 0, st, a->bg, a->W * a->H,
                       out_color, counts);
    GSMPM_LAUNCH_CHECK();
    return GSMPM_OK;
  }
  WsCount* c = nullptr;
  int rc = ws_count(c);
  if (rc) return rc;
  gsmpm_raster r;  // a view of the workspace
  r.forward_only = true;
  r.h_count = c->h;
  r.count_ev = c->ev;
  r.ws = reinterpret_cast<char*>(workspace);
  r.ws_bytes = (size_t)ws_bytes;
  WsWalk w{r.ws, 0};
  rc = ws_pre_walk(w, &r, (size_t)a->P, ntiles);
  if (rc) return rc;
  r.ws_pre = w.off;
  {
    WsWalk probe{nullptr, r.ws_pre};
    gsmpm_raster tmp;
    rc = ws_pairs_walk(probe, &tmp, (size_t)pairs_cap, ntiles);
    if (rc) return rc;
    if (probe.off > r.ws_bytes) {
      set_error("gsmpm_raster_forward_async: the workspace is smaller than gsmpm_raster_workspace_size(P, H, W, "
                "pairs_cap)");
      return GSMPM_ESPACE;
    }
  }
  r.async_cap = pairs_cap;
  r.async_counts = reinterpret_cast<unsigned*>(counts);
  return gsmpm_raster_forward(&r, a, out_color, out_radii, nullptr, stream);
}

int gsmpm_raster_mark_visible(const float* means3D, int32_t P, const float* vm, const float* pm, uint8_t* vis,
                              void* stream) {
  GSMPM_REQUIRE(means3D && vm && vis && P >= 0, "gsmpm_raster_mark_visible: bad argument");
  (void)pm;
  if (P == 0) return GSMPM_OK;
  hipLaunchKernelGGL(k_mark_visible, dim3(div_up(P, 256)), dim3(256), 0, (hipStream_t)stream, means3D, P, vm, vis);
  GSMPM_LAUNCH_CHECK();
  return GSMPM_OK;
}

}  // extern "C"
