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

static void sh_to_rgb(int D, int M, const float* pos, const float* campos, const float* sh, float rgb[3]) {
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

int or_forward(const or_args* a, float* out_color, int32_t* out_radii, float* out_depth, int32_t* out_tt) {
  const int P = a->P, W = a->W, H = a->H;
  const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
  const float fx = W / (2.0f * a->tanfovx), fy = H / (2.0f * a->tanfovy);
  float* xy = (float*)calloc((size_t)P * 2 + 2, sizeof(float));
  float* con = (float*)calloc((size_t)P * 4 + 4, sizeof(float));
  float* rgb = (float*)calloc((size_t)P * 3 + 3, sizeof(float));
  float* depth = (float*)calloc((size_t)P + 1, sizeof(float));
  int32_t* tt = (int32_t*)calloc((size_t)P + 1, sizeof(int32_t));
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
    if (a->colors_precomp == NULL) sh_to_rgb(a->D, a->M, p, a->campos, a->shs + (size_t)i * a->M * 3, rgb + i * 3);
    else memcpy(rgb + i * 3, a->colors_precomp + i * 3, 12);
    depth[i] = pv[2];
    out_radii[i] = rad;
    xy[i * 2] = pt[0]; xy[i * 2 + 1] = pt[1];
    con[i * 4] = conic[0]; con[i * 4 + 1] = conic[1]; con[i * 4 + 2] = conic[2]; con[i * 4 + 3] = a->opacities[i];
    tt[i] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
  }
  long K = 0;
  for (int i = 0; i < P; ++i) K += tt[i];
  kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)(K + 1));
  long off = 0;
  for (int i = 0; i < P; ++i) {
    if (out_radii[i] <= 0) continue;
    int rmin[2], rmax[2];
    get_rect(xy + i * 2, out_radii[i], gx, gy, rmin, rmax);
    uint32_t dbits;
    memcpy(&dbits, &depth[i], 4);
    for (int y = rmin[1]; y < rmax[1]; ++y)
      for (int x = rmin[0]; x < rmax[0]; ++x) {
        kv[off].key = ((uint64_t)(uint32_t)(y * gx + x) << 32) | dbits;
        kv[off].val = (uint32_t)i;
        ++off;
      }
  }
  qsort(kv, (size_t)K, sizeof(kv_t), kv_cmp);
  int ntiles = gx * gy;
  int32_t* rs = (int32_t*)calloc((size_t)ntiles, sizeof(int32_t));
  int32_t* re = (int32_t*)calloc((size_t)ntiles, sizeof(int32_t));
  for (long k = 0; k < K; ++k) {
    int t = (int)(kv[k].key >> 32);
    if (k == 0 || (int)(kv[k - 1].key >> 32) != t) rs[t] = (int32_t)k;
    if (k == K - 1 || (int)(kv[k + 1].key >> 32) != t) re[t] = (int32_t)(k + 1);
  }
  for (int ty = 0; ty < gy; ++ty)
    for (int tx = 0; tx < gx; ++tx) {
      int t = ty * gx + tx;
      for (int py = ty * BY; py < ty * BY + BY && py < H; ++py)
        for (int px = tx * BX; px < tx * BX + BX && px < W; ++px) {
          float T = 1.0f, C[3] = {0, 0, 0};
          float pfx = (float)px, pfy = (float)py;
          for (int k = rs[t]; k < re[t]; ++k) {
            int id = (int)kv[k].val;
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
          }
          for (int ch = 0; ch < 3; ++ch) out_color[(size_t)ch * H * W + (size_t)py * W + px] = C[ch] + T * a->bg[ch];
        }
    }
  if (out_depth) memcpy(out_depth, depth, sizeof(float) * P);
  if (out_tt) memcpy(out_tt, tt, sizeof(int32_t) * P);
  free(xy); free(con); free(rgb); free(depth); free(tt); free(kv); free(rs); free(re);
  return (int)K;
}
