/*
 * raster_oracle.c -- scalar C restatement of the 3DGS rasterizer forward.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Third-party algorithm: graphdeco-inria/diff-gaussian-rasterization, forward
 * pass of the pre-2024 API (2-tuple return), which the reference calls at
 * main.py:16,118-156 but does not vendor.  Restated
 * from the public algorithm: preprocessCUDA -> inclusive scan ->
 * duplicateWithKeys -> stable radix sort on (tile<<32 | depth bits) ->
 * identifyTileRanges -> renderCUDA.  "Parity unpinned" against upstream:
 * this restatement is pinned by analytic KATs (tests/test_oracle_kat.py).
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define BX 16
#define BY 16

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

static inline float mxf(float a, float b) { return a > b ? a : b; }
static inline float mnf(float a, float b) { return a < b ? a : b; }
static inline int mxi(int a, int b) { return a > b ? a : b; }
static inline int mni(int a, int b) { return a < b ? a : b; }

static void xform4x3(const float* p, const float* m, float* o) {
  o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
  o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
  o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static void xform4x4(const float* p, const float* m, float* o) {
  xform4x3(p, m, o);
  o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}
static float ndc2pix(float v, int S) { return ((v + 1.0f) * S - 1.0f) * 0.5f; }

static void get_rect(const float pt[2], int r, int gx, int gy, int rmin[2], int rmax[2]) {
  rmin[0] = mni(gx, mxi(0, (int)((pt[0] - r) / BX)));
  rmin[1] = mni(gy, mxi(0, (int)((pt[1] - r) / BY)));
  rmax[0] = mni(gx, mxi(0, (int)((pt[0] + r + BX - 1) / BX)));
  rmax[1] = mni(gy, mxi(0, (int)((pt[1] + r + BY - 1) / BY)));
}

/* computeCov3D: Sigma = (S R)^T (S R) in glm's column-major convention */
static void cov3d_from_sr(const float* s, float mod, const float* rot, float* c6) {
  float S[3] = {mod * s[0], mod * s[1], mod * s[2]};
  float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
  /* R (math, row-major) = standard quaternion rotation */
  float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
  /* M = R diag(S) ; Sigma = M M^T */
  float M[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[i * 3 + j] = R[i * 3 + j] * S[j];
  float Sg[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Sg[i * 3 + j] = M[i * 3 + 0] * M[j * 3 + 0] + M[i * 3 + 1] * M[j * 3 + 1] + M[i * 3 + 2] * M[j * 3 + 2];
  c6[0] = Sg[0]; c6[1] = Sg[1]; c6[2] = Sg[2]; c6[3] = Sg[4]; c6[4] = Sg[5]; c6[5] = Sg[8];
}

/* computeCov2D (EWA splatting, Zwicker et al.) */
static void cov2d(const float* mean, float fx, float fy, float tanx, float tany, const float* c3, const float* vm, float out[3]) {
  float t[3];
  xform4x3(mean, vm, t);
  const float limx = 1.3f * tanx, limy = 1.3f * tany;
  const float txtz = t[0] / t[2], tytz = t[1] / t[2];
  t[0] = mnf(limx, mxf(-limx, txtz)) * t[2];
  t[1] = mnf(limy, mxf(-limy, tytz)) * t[2];
  /* J (2 rows used), math layout */
  float J00 = fx / t[2], J02 = -(fx * t[0]) / (t[2] * t[2]);
  float J11 = fy / t[2], J12 = -(fy * t[1]) / (t[2] * t[2]);
  /* W = rotation part of world->view, math row-major: W[r][c] = vm[c*4 + r] */
  float W[9] = {vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]};
  /* T = J W (2x3) */
  float T[2][3];
  for (int c = 0; c < 3; ++c) {
    T[0][c] = J00 * W[0 * 3 + c] + J02 * W[2 * 3 + c];
    T[1][c] = J11 * W[1 * 3 + c] + J12 * W[2 * 3 + c];
  }
  float V[9] = {c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]};
  float TV[2][3];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 3; ++c) TV[r][c] = T[r][0] * V[0 * 3 + c] + T[r][1] * V[1 * 3 + c] + T[r][2] * V[2 * 3 + c];
  float a = TV[0][0] * T[0][0] + TV[0][1] * T[0][1] + TV[0][2] * T[0][2];
  float b = TV[0][0] * T[1][0] + TV[0][1] * T[1][1] + TV[0][2] * T[1][2];
  float c = TV[1][0] * T[1][0] + TV[1][1] * T[1][1] + TV[1][2] * T[1][2];
  out[0] = a + 0.3f;
  out[1] = b;
  out[2] = c + 0.3f;
}

static void sh_to_rgb(int D, int M, const float* pos, const float* campos, const float* sh, float rgb[3],
                      uint8_t clamped[3]) {
  float dir[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
  float len = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
  dir[0] /= len; dir[1] /= len; dir[2] /= len;
  (void)M;
  for (int ch = 0; ch < 3; ++ch) {
#define SHC(k) sh[(k) * 3 + ch]
    float r = SH_C0 * SHC(0);
    if (D > 0) {
      float x = dir[0], y = dir[1], z = dir[2];
      r = r - SH_C1 * y * SHC(1) + SH_C1 * z * SHC(2) - SH_C1 * x * SHC(3);
      if (D > 1) {
        float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        r = r + SH_C2[0] * xy * SHC(4) + SH_C2[1] * yz * SHC(5) + SH_C2[2] * (2.0f * zz - xx - yy) * SHC(6) +
            SH_C2[3] * xz * SHC(7) + SH_C2[4] * (xx - yy) * SHC(8);
        if (D > 2) {
          r = r + SH_C3[0] * y * (3.0f * xx - yy) * SHC(9) + SH_C3[1] * xy * z * SHC(10) +
              SH_C3[2] * y * (4.0f * zz - xx - yy) * SHC(11) + SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * SHC(12) +
              SH_C3[4] * x * (4.0f * zz - xx - yy) * SHC(13) + SH_C3[5] * z * (xx - yy) * SHC(14) +
              SH_C3[6] * x * (xx - 3.0f * yy) * SHC(15);
        }
      }
    }
#undef SHC
    r += 0.5f;
    clamped[ch] = r < 0.0f;
    rgb[ch] = mxf(r, 0.0f);
  }
}

typedef struct { uint64_t key; uint32_t val; } kv_t;
static int kv_cmp(const void* a, const void* b) {
  const kv_t* x = (const kv_t*)a; const kv_t* y = (const kv_t*)b;
  if (x->key < y->key) return -1;
  if (x->key > y->key) return 1;
  return x->val < y->val ? -1 : (x->val > y->val ? 1 : 0); /* == stable by emission order */
}

/* Forward state kept for the backward pass (upstream's geom/binning/image buffers). */
typedef struct {
  int P, W, H, gx, gy;
  float fx, fy;
  float *xy, *con, *rgb, *depth;
  uint8_t* clamped;
  int32_t *radii, *tt, *rs, *re;
  kv_t* kv;
  long K;
  float* final_T;     /* [H*W] */
  int32_t* n_contrib; /* [H*W] */
} fstate;

static void fs_free(fstate* f) {
  free(f->xy); free(f->con); free(f->rgb); free(f->depth); free(f->clamped); free(f->radii); free(f->tt);
  free(f->rs); free(f->re); free(f->kv); free(f->final_T); free(f->n_contrib);
}

/* crop (test infrastructure for large frames): only the pairs of tiles
 * [c[0], c[2]) x [c[1], c[3]) are emitted, sorted and blended -- the same
 * per-tile lists as the full frame (a tile's list is its own pairs in
 * (depth, index) order); preprocess, radii, tiles_touched and K stay global.
 * NULL: the whole frame. */
static void forward_core(const or_args* a, fstate* f, float* out_color, const int* crop) {
  const int P = a->P, W = a->W, H = a->H;
  const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
  const int cx0 = crop ? mxi(0, crop[0]) : 0, cy0 = crop ? mxi(0, crop[1]) : 0;
  const int cx1 = crop ? mni(gx, crop[2]) : gx, cy1 = crop ? mni(gy, crop[3]) : gy;
  const float fx = W / (2.0f * a->tanfovx), fy = H / (2.0f * a->tanfovy);
  f->P = P; f->W = W; f->H = H; f->gx = gx; f->gy = gy; f->fx = fx; f->fy = fy;
  float* xy = f->xy = (float*)calloc((size_t)P * 2 + 2, sizeof(float));
  float* con = f->con = (float*)calloc((size_t)P * 4 + 4, sizeof(float));
  float* rgb = f->rgb = (float*)calloc((size_t)P * 3 + 3, sizeof(float));
  float* depth = f->depth = (float*)calloc((size_t)P + 1, sizeof(float));
  uint8_t* clamped = f->clamped = (uint8_t*)calloc((size_t)P * 3 + 3, 1);
  int32_t* tt = f->tt = (int32_t*)calloc((size_t)P + 1, sizeof(int32_t));
  int32_t* out_radii = f->radii = (int32_t*)calloc((size_t)P + 1, sizeof(int32_t));
  f->final_T = (float*)calloc((size_t)W * H, sizeof(float));
  f->n_contrib = (int32_t*)calloc((size_t)W * H, sizeof(int32_t));
  for (int i = 0; i < P; ++i) {
    out_radii[i] = 0;
    const float* p = a->means3D + i * 3;
    float pv[3];
    xform4x3(p, a->viewmatrix, pv);
    if (pv[2] <= 0.2f) continue; /* in_frustum */
    float ph[4];
    xform4x4(p, a->projmatrix, ph);
    float pw = 1.0f / (ph[3] + 0.0000001f);
    float pp[3] = {ph[0] * pw, ph[1] * pw, ph[2] * pw};
    float c6[6];
    const float* c3;
    if (a->cov3D_precomp) c3 = a->cov3D_precomp + i * 6;
    else { cov3d_from_sr(a->scales + i * 3, a->scale_modifier, a->rotations + i * 4, c6); c3 = c6; }
    float cv[3];
    cov2d(p, fx, fy, a->tanfovx, a->tanfovy, c3, a->viewmatrix, cv);
    float det = cv[0] * cv[2] - cv[1] * cv[1];
    if (det == 0.0f) continue;
    float di = 1.f / det;
    float conic[3] = {cv[2] * di, -cv[1] * di, cv[0] * di};
    float mid = 0.5f * (cv[0] + cv[2]);
    float l1 = mid + sqrtf(mxf(0.1f, mid * mid - det));
    float l2 = mid - sqrtf(mxf(0.1f, mid * mid - det));
    int rad = (int)ceilf(3.f * sqrtf(mxf(l1, l2)));
    float pt[2] = {ndc2pix(pp[0], W), ndc2pix(pp[1], H)};
    int rmin[2], rmax[2];
    get_rect(pt, rad, gx, gy, rmin, rmax);
    if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
    if (a->colors_precomp == NULL)
      sh_to_rgb(a->D, a->M, p, a->campos, a->shs + (size_t)i * a->M * 3, rgb + i * 3, clamped + i * 3);
    else memcpy(rgb + i * 3, a->colors_precomp + i * 3, 12);
    depth[i] = pv[2];
    out_radii[i] = rad;
    xy[i * 2] = pt[0]; xy[i * 2 + 1] = pt[1];
    con[i * 4] = conic[0]; con[i * 4 + 1] = conic[1]; con[i * 4 + 2] = conic[2]; con[i * 4 + 3] = a->opacities[i];
    tt[i] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
  }
  long K = 0, Kc = 0;
  for (int i = 0; i < P; ++i) {
    K += tt[i];
    if (out_radii[i] <= 0 || !crop) continue;
    int rmin[2], rmax[2];
    get_rect(xy + i * 2, out_radii[i], gx, gy, rmin, rmax);
    const long wx = mni(rmax[0], cx1) - mxi(rmin[0], cx0), wy = mni(rmax[1], cy1) - mxi(rmin[1], cy0);
    if (wx > 0 && wy > 0) Kc += wx * wy;
  }
  if (!crop) Kc = K;
  kv_t* kv = f->kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)(Kc + 1));
  f->K = K;
  /* The sorted pair list of upstream's stable radix sort on (tile << 32 |
   * depth bits), built tile by tile: count each tile's pairs, place every
   * Gaussian's pairs into its tiles' runs in index order, then sort each run
   * by (depth bits, index) -- the same order as one global sort on (key,
   * emission index), since a Gaussian's pairs in one tile are one pair.  The
   * per-tile runs sort independently (OpenMP build: in parallel; the serial
   * checker gives the same array). */
  int ntiles = gx * gy;
  int32_t* rs = f->rs = (int32_t*)calloc((size_t)ntiles, sizeof(int32_t));
  int32_t* re = f->re = (int32_t*)calloc((size_t)ntiles, sizeof(int32_t));
  long* tcur = (long*)calloc((size_t)ntiles + 1, sizeof(long));
  for (int i = 0; i < P; ++i) {
    if (out_radii[i] <= 0) continue;
    int rmin[2], rmax[2];
    get_rect(xy + i * 2, out_radii[i], gx, gy, rmin, rmax);
    for (int y = mxi(rmin[1], cy0); y < mni(rmax[1], cy1); ++y)
      for (int x = mxi(rmin[0], cx0); x < mni(rmax[0], cx1); ++x) tcur[y * gx + x + 1] += 1;
  }
  for (int t = 0; t < ntiles; ++t) {
    tcur[t + 1] += tcur[t];
    rs[t] = (int32_t)tcur[t];
    re[t] = (int32_t)tcur[t + 1];
  }
  for (int i = 0; i < P; ++i) {
    if (out_radii[i] <= 0) continue;
    int rmin[2], rmax[2];
    get_rect(xy + i * 2, out_radii[i], gx, gy, rmin, rmax);
    uint32_t dbits;
    memcpy(&dbits, &depth[i], 4);
    for (int y = mxi(rmin[1], cy0); y < mni(rmax[1], cy1); ++y)
      for (int x = mxi(rmin[0], cx0); x < mni(rmax[0], cx1); ++x) {
        const long o = tcur[y * gx + x]++;
        kv[o].key = ((uint64_t)(uint32_t)(y * gx + x) << 32) | dbits;
        kv[o].val = (uint32_t)i;
      }
  }
  free(tcur);
#pragma omp parallel for schedule(dynamic, 16)
  for (int t = 0; t < ntiles; ++t)
    if (re[t] - rs[t] > 1) qsort(kv + rs[t], (size_t)(re[t] - rs[t]), sizeof(kv_t), kv_cmp);
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
  for (int ty = cy0; ty < cy1; ++ty)
    for (int tx = cx0; tx < cx1; ++tx) {
      int t = ty * gx + tx;
      for (int py = ty * BY; py < ty * BY + BY && py < H; ++py)
        for (int px = tx * BX; px < tx * BX + BX && px < W; ++px) {
          float T = 1.0f, C[3] = {0, 0, 0};
          float pfx = (float)px, pfy = (float)py;
          int contributor = 0, last = 0;
          for (int k = rs[t]; k < re[t]; ++k) {
            int id = (int)kv[k].val;
            ++contributor;
            float dxp = xy[id * 2] - pfx, dyp = xy[id * 2 + 1] - pfy;
            const float* co = con + id * 4;
            float power = -0.5f * (co[0] * dxp * dxp + co[2] * dyp * dyp) - co[1] * dxp * dyp;
            if (power > 0.0f) continue;
            float alpha = mnf(0.99f, co[3] * expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            float test_T = T * (1 - alpha);
            if (test_T < 0.0001f) break;
            for (int ch = 0; ch < 3; ++ch) C[ch] += rgb[id * 3 + ch] * alpha * T;
            T = test_T;
            last = contributor;
          }
          const size_t pix = (size_t)py * W + px;
          f->final_T[pix] = T;
          f->n_contrib[pix] = last;
          if (out_color)
            for (int ch = 0; ch < 3; ++ch) out_color[(size_t)ch * H * W + pix] = C[ch] + T * a->bg[ch];
        }
    }
}

int or_forward(const or_args* a, float* out_color, int32_t* out_radii, float* out_depth, int32_t* out_tt) {
  return or_forward_crop(a, out_color, out_radii, out_depth, out_tt, NULL);
}

long or_forward_crop(const or_args* a, float* out_color, int32_t* out_radii, float* out_depth, int32_t* out_tt,
                     const int* crop4) {
  fstate f;
  forward_core(a, &f, out_color, crop4);
  memcpy(out_radii, f.radii, sizeof(int32_t) * a->P);
  if (out_depth) memcpy(out_depth, f.depth, sizeof(float) * a->P);
  if (out_tt) memcpy(out_tt, f.tt, sizeof(int32_t) * a->P);
  const long K = f.K;
  fs_free(&f);
  return K;
}

/* ------------------------------------------------------------ backward ---
 * Restates upstream's BACKWARD::render / computeCov2DCUDA / preprocessCUDA
 * (computeColorFromSH, computeCov3D backward) of the same pre-2024 API.  The
 * derivatives are the chain rule of the forward above, with upstream's
 * deviations from the exact derivative kept:
 *   - alpha = min(0.99, o G): the gradient ignores the clamp;
 *   - the 1.3 x fov clamp of t: dt.x (dt.y) is zeroed when clamped, and the
 *     t.z term uses the clamped t.x (t.y) without its t.z dependence;
 *   - the conic gradient's 1/(det^2 + 1e-7);
 *   - the scale gradient is w.r.t. scale_modifier * scale.
 * dL_dmeans2D is w.r.t. the NDC position (pixel offsets scaled by W/2, H/2).
 */
static void dnormvdv(const float v[3], const float dv[3], float out[3]) {
  const float sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
  out[0] = ((sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
  out[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
  out[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* d rgb / d (sh, dir) for one Gaussian: dL_dsh (+=), dL_dmean (+=) */
static void sh_backward(int D, const float* pos, const float* campos, const float* sh, const uint8_t clamped[3],
                        const float dL_dcolor[3], float* dL_dsh, float dL_dmean[3]) {
  const float dir_orig[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
  const float len = sqrtf(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
  const float x = dir_orig[0] / len, y = dir_orig[1] / len, z = dir_orig[2] / len;
  float g[3];
  for (int ch = 0; ch < 3; ++ch) g[ch] = clamped[ch] ? 0.f : dL_dcolor[ch];
  float dRdx[3] = {0, 0, 0}, dRdy[3] = {0, 0, 0}, dRdz[3] = {0, 0, 0};
#define SHC(k, ch) sh[(k) * 3 + (ch)]
#define DSH(k, coef) for (int ch = 0; ch < 3; ++ch) dL_dsh[(k) * 3 + ch] += (coef) * g[ch]
  DSH(0, SH_C0);
  if (D > 0) {
    DSH(1, -SH_C1 * y);
    DSH(2, SH_C1 * z);
    DSH(3, -SH_C1 * x);
    for (int ch = 0; ch < 3; ++ch) {
      dRdx[ch] = -SH_C1 * SHC(3, ch);
      dRdy[ch] = -SH_C1 * SHC(1, ch);
      dRdz[ch] = SH_C1 * SHC(2, ch);
    }
    if (D > 1) {
      const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      DSH(4, SH_C2[0] * xy);
      DSH(5, SH_C2[1] * yz);
      DSH(6, SH_C2[2] * (2.f * zz - xx - yy));
      DSH(7, SH_C2[3] * xz);
      DSH(8, SH_C2[4] * (xx - yy));
      for (int ch = 0; ch < 3; ++ch) {
        dRdx[ch] += SH_C2[0] * y * SHC(4, ch) + SH_C2[2] * 2.f * -x * SHC(6, ch) + SH_C2[3] * z * SHC(7, ch) +
                    SH_C2[4] * 2.f * x * SHC(8, ch);
        dRdy[ch] += SH_C2[0] * x * SHC(4, ch) + SH_C2[1] * z * SHC(5, ch) + SH_C2[2] * 2.f * -y * SHC(6, ch) +
                    SH_C2[4] * 2.f * -y * SHC(8, ch);
        dRdz[ch] += SH_C2[1] * y * SHC(5, ch) + SH_C2[2] * 2.f * 2.f * z * SHC(6, ch) + SH_C2[3] * x * SHC(7, ch);
      }
      if (D > 2) {
        DSH(9, SH_C3[0] * y * (3.f * xx - yy));
        DSH(10, SH_C3[1] * xy * z);
        DSH(11, SH_C3[2] * y * (4.f * zz - xx - yy));
        DSH(12, SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy));
        DSH(13, SH_C3[4] * x * (4.f * zz - xx - yy));
        DSH(14, SH_C3[5] * z * (xx - yy));
        DSH(15, SH_C3[6] * x * (xx - 3.f * yy));
        for (int ch = 0; ch < 3; ++ch) {
          dRdx[ch] += SH_C3[0] * SHC(9, ch) * 3.f * 2.f * xy + SH_C3[1] * SHC(10, ch) * yz +
                      SH_C3[2] * SHC(11, ch) * -2.f * xy + SH_C3[3] * SHC(12, ch) * -3.f * 2.f * xz +
                      SH_C3[4] * SHC(13, ch) * (-3.f * xx + 4.f * zz - yy) + SH_C3[5] * SHC(14, ch) * 2.f * xz +
                      SH_C3[6] * SHC(15, ch) * 3.f * (xx - yy);
          dRdy[ch] += SH_C3[0] * SHC(9, ch) * 3.f * (xx - yy) + SH_C3[1] * SHC(10, ch) * xz +
                      SH_C3[2] * SHC(11, ch) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * SHC(12, ch) * -3.f * 2.f * yz +
                      SH_C3[4] * SHC(13, ch) * -2.f * xy + SH_C3[5] * SHC(14, ch) * -2.f * yz +
                      SH_C3[6] * SHC(15, ch) * -3.f * 2.f * xy;
          dRdz[ch] += SH_C3[1] * SHC(10, ch) * xy + SH_C3[2] * SHC(11, ch) * 4.f * 2.f * yz +
                      SH_C3[3] * SHC(12, ch) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * SHC(13, ch) * 4.f * 2.f * xz +
                      SH_C3[5] * SHC(14, ch) * (xx - yy);
        }
      }
    }
  }
#undef SHC
#undef DSH
  const float dL_ddir[3] = {dRdx[0] * g[0] + dRdx[1] * g[1] + dRdx[2] * g[2],
                            dRdy[0] * g[0] + dRdy[1] * g[1] + dRdy[2] * g[2],
                            dRdz[0] * g[0] + dRdz[1] * g[1] + dRdz[2] * g[2]};
  float dm[3];
  dnormvdv(dir_orig, dL_ddir, dm);
  for (int d = 0; d < 3; ++d) dL_dmean[d] += dm[d];
}

/* computeCov3D backward: dL_dcov6 -> dL_dscale (w.r.t. mod * scale), dL_drot (unnormalised q) */
static void cov3d_backward(const float* s, float mod, const float* rot, const float* dc, float dL_ds[3], float dL_dq[4]) {
  const float S[3] = {mod * s[0], mod * s[1], mod * s[2]};
  const float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
  const float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                      2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                      2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
  /* symmetric dL/dSigma: stored off-diagonal gradients split over both entries */
  const float G[9] = {dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2], 0.5f * dc[4], dc[5]};
  float M[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[i * 3 + j] = R[i * 3 + j] * S[j];
  /* Sigma = M M^T -> dL/dM = 2 G M */
  float dM[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dM[i * 3 + j] = 2.f * (G[i * 3 + 0] * M[0 * 3 + j] + G[i * 3 + 1] * M[1 * 3 + j] + G[i * 3 + 2] * M[2 * 3 + j]);
  float dR[9];
  for (int j = 0; j < 3; ++j) {
    dL_ds[j] = dM[0 * 3 + j] * R[0 * 3 + j] + dM[1 * 3 + j] * R[1 * 3 + j] + dM[2 * 3 + j] * R[2 * 3 + j];
    for (int i = 0; i < 3; ++i) dR[i * 3 + j] = dM[i * 3 + j] * S[j];
  }
  /* R(q) entries -> q = (r, x, y, z) */
  dL_dq[0] = 2.f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
  dL_dq[1] = 2.f * (y * dR[1] + z * dR[2] + y * dR[3] - 2.f * x * dR[4] - r * dR[5] + z * dR[6] + r * dR[7] - 2.f * x * dR[8]);
  dL_dq[2] = 2.f * (-2.f * y * dR[0] + x * dR[1] + r * dR[2] + x * dR[3] + z * dR[5] - r * dR[6] + z * dR[7] - 2.f * y * dR[8]);
  dL_dq[3] = 2.f * (-2.f * z * dR[0] - r * dR[1] + x * dR[2] + r * dR[3] - 2.f * z * dR[4] + y * dR[5] + x * dR[6] + y * dR[7]);
}

void or_backward(const or_args* a, const float* dL_dpix, float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity,
                 float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drot) {
  const int P = a->P, W = a->W, H = a->H;
  fstate f;
  forward_core(a, &f, NULL, NULL);
  float* dconic = (float*)calloc((size_t)P * 3 + 3, sizeof(float));
  memset(dL_dmeans2D, 0, sizeof(float) * 3 * P);
  memset(dL_dcolors, 0, sizeof(float) * 3 * P);
  memset(dL_dopacity, 0, sizeof(float) * P);
  memset(dL_dmeans3D, 0, sizeof(float) * 3 * P);
  memset(dL_dcov3D, 0, sizeof(float) * 6 * P);
  if (dL_dsh) memset(dL_dsh, 0, sizeof(float) * 3 * (size_t)a->M * P);
  if (dL_dscales) memset(dL_dscales, 0, sizeof(float) * 3 * P);
  if (dL_drot) memset(dL_drot, 0, sizeof(float) * 4 * P);
  const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
  /* BACKWARD::render: per pixel, back to front from the last contributor */
  for (int ty = 0; ty < f.gy; ++ty)
    for (int tx = 0; tx < f.gx; ++tx) {
      const int t = ty * f.gx + tx;
      for (int py = ty * BY; py < ty * BY + BY && py < H; ++py)
        for (int px = tx * BX; px < tx * BX + BX && px < W; ++px) {
          const size_t pix = (size_t)py * W + px;
          const float T_final = f.final_T[pix];
          float T = T_final;
          const int last = f.n_contrib[pix];
          float dpx[3], accum[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, last_alpha = 0.f;
          for (int ch = 0; ch < 3; ++ch) dpx[ch] = dL_dpix[(size_t)ch * H * W + pix];
          const float bg_dot = a->bg[0] * dpx[0] + a->bg[1] * dpx[1] + a->bg[2] * dpx[2];
          for (int k = f.re[t] - 1; k >= f.rs[t]; --k) {
            if (k - f.rs[t] >= last) continue;
            const int id = (int)f.kv[k].val;
            const float dx = f.xy[id * 2] - (float)px, dy = f.xy[id * 2 + 1] - (float)py;
            const float* co = f.con + id * 4;
            const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
            if (power > 0.0f) continue;
            const float G = expf(power);
            const float alpha = mnf(0.99f, co[3] * G);
            if (alpha < 1.0f / 255.0f) continue;
            T = T / (1.f - alpha);
            const float dchannel_dcolor = alpha * T;
            float dL_dalpha = 0.f;
            for (int ch = 0; ch < 3; ++ch) {
              const float c = f.rgb[id * 3 + ch];
              accum[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum[ch];
              last_color[ch] = c;
              dL_dalpha += (c - accum[ch]) * dpx[ch];
              dL_dcolors[id * 3 + ch] += dchannel_dcolor * dpx[ch];
            }
            dL_dalpha *= T;
            last_alpha = alpha;
            dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
            const float dL_dG = co[3] * dL_dalpha;
            const float gdx = G * dx, gdy = G * dy;
            const float dG_ddelx = -gdx * co[0] - gdy * co[1];
            const float dG_ddely = -gdy * co[2] - gdx * co[1];
            dL_dmeans2D[id * 3 + 0] += dL_dG * dG_ddelx * ddelx_dx;
            dL_dmeans2D[id * 3 + 1] += dL_dG * dG_ddely * ddely_dy;
            dconic[id * 3 + 0] += -0.5f * gdx * dx * dL_dG;
            dconic[id * 3 + 1] += -0.5f * gdx * dy * dL_dG;
            dconic[id * 3 + 2] += -0.5f * gdy * dy * dL_dG;
            dL_dopacity[id] += G * dL_dalpha;
          }
        }
    }
  /* computeCov2DCUDA backward + preprocessCUDA backward, per Gaussian with radius > 0 */
  for (int i = 0; i < P; ++i) {
    if (!(f.radii[i] > 0)) continue;
    const float* m = a->means3D + i * 3;
    float c6[6];
    const float* c3;
    if (a->cov3D_precomp) c3 = a->cov3D_precomp + i * 6;
    else { cov3d_from_sr(a->scales + i * 3, a->scale_modifier, a->rotations + i * 4, c6); c3 = c6; }
    const float* vm = a->viewmatrix;
    float t[3];
    xform4x3(m, vm, t);
    const float limx = 1.3f * a->tanfovx, limy = 1.3f * a->tanfovy;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = mnf(limx, mxf(-limx, txtz)) * t[2];
    t[1] = mnf(limy, mxf(-limy, tytz)) * t[2];
    const float x_mul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    const float y_mul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const float hx = f.fx, hy = f.fy;
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
    const float* dco = dconic + i * 3;
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    float* dcov = dL_dcov3D + i * 6;
    if (denom2inv != 0.f) {
      dL_da = denom2inv * (-cc * cc * dco[0] + 2.f * cb * cc * dco[1] + (denom - ca * cc) * dco[2]);
      dL_dc = denom2inv * (-ca * ca * dco[2] + 2.f * ca * cb * dco[1] + (denom - ca * cc) * dco[0]);
      dL_db = denom2inv * 2.f * (cb * cc * dco[0] - (denom + 2.f * cb * cb) * dco[1] + ca * cb * dco[2]);
      const int di[6] = {0, 0, 0, 1, 1, 2}, dj[6] = {0, 1, 2, 1, 2, 2};
      for (int e = 0; e < 6; ++e) {
        const int p = di[e], q = dj[e];
        if (p == q) dcov[e] = T0[p] * T0[p] * dL_da + T0[p] * T1[p] * dL_db + T1[p] * T1[p] * dL_dc;
        else dcov[e] = 2.f * T0[p] * T0[q] * dL_da + (T0[p] * T1[q] + T0[q] * T1[p]) * dL_db + 2.f * T1[p] * T1[q] * dL_dc;
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
    float* dm = dL_dmeans3D + i * 3;
    dm[0] = vm[0] * dtx + vm[1] * dty + vm[2] * dtz;
    dm[1] = vm[4] * dtx + vm[5] * dty + vm[6] * dtz;
    dm[2] = vm[8] * dtx + vm[9] * dty + vm[10] * dtz;
    /* projection of the mean */
    const float* pm = a->projmatrix;
    float mh[4];
    xform4x4(m, pm, mh);
    const float mw = 1.0f / (mh[3] + 0.0000001f);
    const float mul1 = (pm[0] * m[0] + pm[4] * m[1] + pm[8] * m[2] + pm[12]) * mw * mw;
    const float mul2 = (pm[1] * m[0] + pm[5] * m[1] + pm[9] * m[2] + pm[13]) * mw * mw;
    const float g2x = dL_dmeans2D[i * 3 + 0], g2y = dL_dmeans2D[i * 3 + 1];
    dm[0] += (pm[0] * mw - pm[3] * mul1) * g2x + (pm[1] * mw - pm[3] * mul2) * g2y;
    dm[1] += (pm[4] * mw - pm[7] * mul1) * g2x + (pm[5] * mw - pm[7] * mul2) * g2y;
    dm[2] += (pm[8] * mw - pm[11] * mul1) * g2x + (pm[9] * mw - pm[11] * mul2) * g2y;
    if (a->shs && dL_dsh)
      sh_backward(a->D, m, a->campos, a->shs + (size_t)i * a->M * 3, f.clamped + i * 3, dL_dcolors + i * 3,
                  dL_dsh + (size_t)i * a->M * 3, dm);
    if (a->scales && dL_dscales && dL_drot)
      cov3d_backward(a->scales + i * 3, a->scale_modifier, a->rotations + i * 4, dcov, dL_dscales + i * 3, dL_drot + i * 4);
  }
  free(dconic);
  fs_free(&f);
}
