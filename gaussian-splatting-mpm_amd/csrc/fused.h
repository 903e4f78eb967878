// fused.h -- the default substep pipeline of libgsmpm (included by mpm.hip
// inside namespace gsmpm, after the per-phase kernels it shares helpers with).
//
// The reference runs every substep as stress -> p2g -> grid -> g2p
// (mpm_solver/solver.py:27-52).  Here G2P of substep s and P2G of substep
// s + 1 run in ONE kernel, `k_fused`, so a substep is two launches
// (k_fused, k_grid_f) instead of four:
//
//   k_fused   one workgroup per <= 256-particle chunk of a tile: stage the
//             tile's v_out window in LDS, gather (g2p, utils.py:218-282),
//             then -- with x, v, C, F_trial still in registers -- impulse,
//             return map + stress (utils.py:13-54) and the APIC scatter
//             (p2g, utils.py:89-134) into the chunk's 64-bit fixed-point LDS
//             window, stored to the chunk's slot
//   k_grid_f  one workgroup per touched tile: sum the covering chunk windows
//             (fixed order), normalise + gravity + BC list -> v_out
//
// Particles keep the chunk (tile) they were binned into for `rebin_interval`
// substeps, so a chunk's window must hold the stencils of particles that
// moved since the binning: the window is the tile plus a ONE-cell margin on
// every side (base cell in [o - 1, o + T], nodes [o - 1, o + T + 3)).  With
// tiles of 8 x 8 x 7 cells that is 12 x 12 x 11 = 1584 nodes, 50.7 KB of u64
// accumulators -- three workgroups per CU.  A particle that moved further
// gathers from the dense v_out and scatters with global float atomics into
// the dense accumulator, and raises the escape flag that makes the next grid
// update sweep every tile (correct for any motion, fast for CFL-bounded
// motion; the lego scene moves < 0.06 cells per substep).
//
// Binning is done by the G2P half of k_fused every `rebin_interval` substeps
// (counts + touched flags), `k_finish_bins` turns the counts into chunk
// records, exactly as in the per-phase pipeline.

#ifndef GSMPM_FT2
#define GSMPM_FT2 7
#endif
constexpr int kFT0 = 8, kFT1 = 8, kFT2 = GSMPM_FT2;          // tile cells per axis
constexpr int kFW0 = kFT0 + 4, kFW1 = kFT1 + 4, kFW2 = kFT2 + 4;  // window nodes per axis
constexpr int kFWin = kFW0 * kFW1 * kFW2;                      // 1584
constexpr int kFTN = kFT0 * kFT1 * kFT2;                       // owned nodes per tile (448)

// Where window node (w0, w1, w2) lives in its chunk's slot.  Default: window
// order ([kFW0][kFW1][kFW2]).  GSMPM_OWNER_SLOTS=1 (A/B): grouped by the tile
// that owns the node -- per axis the window's coords split into sections
// w = 0 (the lower neighbour's last plane), 1..T (the tile's own), T+1..T+3
// (the upper neighbour's first three), and the 27 section boxes are stored
// one after another, each in its owner tile's node order.  A grid-update wave
// (64 consecutive owned nodes of one tile) then reads the own tile's box and
// the lower-x neighbour's as one contiguous 1 KB run instead of 9 runs of 7
// nodes 11 apart.
#ifndef GSMPM_OWNER_SLOTS
#define GSMPM_OWNER_SLOTS 0
#endif
constexpr bool kOwnerSlots = GSMPM_OWNER_SLOTS != 0;
__device__ __forceinline__ int slot_sec_pre(int w, int T) { return w == 0 ? 0 : (w <= T ? 1 : T + 1); }
__device__ __forceinline__ int slot_sec_n(int w, int T) { return w == 0 ? 1 : (w <= T ? T : 3); }
__device__ __forceinline__ int slot_loc(int w0, int w1, int w2) {
  if constexpr (!kOwnerSlots) {
    return (w0 * kFW1 + w1) * kFW2 + w2;
  } else {
    const int p0 = slot_sec_pre(w0, kFT0), n0 = slot_sec_n(w0, kFT0);
    const int p1 = slot_sec_pre(w1, kFT1), n1 = slot_sec_n(w1, kFT1);
    const int p2 = slot_sec_pre(w2, kFT2), n2 = slot_sec_n(w2, kFT2);
    return p0 * (kFW1 * kFW2) + n0 * (p1 * kFW2 + n1 * p2) + ((w0 - p0) * n1 + (w1 - p1)) * n2 + (w2 - p2);
  }
}

// ---- multi-GPU slab hooks (slab.h has the exchange and migration kernels) ----
struct SlabWin {
  int W;            // window planes (0: not a slab)
  int a[2];         // first plane of the lower (0) / upper (1) window; window w is [a[w], a[w] + W)
  int on[2];        // window w present (a neighbour on that side)
  float4* part[2];  // [W][ny][nz] this rank's partial sums of the window's nodes in its rect (k_grid_f writes,
                    // k_win_update zeroes)
  int y0[2], ny[2];  // window w's rect of nodes [y0, y0 + ny) x [z0, z0 + nz): what the two ranks of the bound can
  int z0[2], nz[2];  // touch before the next migration (agreed at every migration); only it is exchanged
  int* oob;          // set when a window node outside the rect has mass (the exchange would miss it)
  int pass;          // k_grid_f: 0 every touched tile, 1 tiles meeting a window, 2 the others
};

__device__ __forceinline__ int slab_window_of(const SlabWin& sw, int i) {
  if (sw.on[0] && i >= sw.a[0] && i < sw.a[0] + sw.W) return 0;
  if (sw.on[1] && i >= sw.a[1] && i < sw.a[1] + sw.W) return 1;
  return -1;
}
// does tile-x ti (planes [ti * kFT0, ti * kFT0 + kFT0)) meet a window?
__device__ __forceinline__ bool slab_tile_in_window(const SlabWin& sw, int ti) {
  const int p0 = ti * kFT0, p1 = p0 + kFT0;
  bool r = false;
#pragma unroll
  for (int w = 0; w < 2; ++w) r = r || (sw.on[w] && p0 < sw.a[w] + sw.W && sw.a[w] < p1);
  return r;
}

// per-particle checks of k_fused: the slab drift check (base plane allowed in
// [xlo, xhi), else *FusedRare::drift) and the non-finite check (a
// NaN / Inf position sets *FusedRare::nonfin, which the step call reports as
// GSMPM_ESTATE; without it a non-finite particle is silently binned
// "outside" and scatters nowhere)
__device__ __forceinline__ bool finite3(const float (&x)[3]) {
  return __builtin_isfinite(x[0]) && __builtin_isfinite(x[1]) && __builtin_isfinite(x[2]);
}

struct FTiles {
  int td0, td1, td2;  // tiles per axis
  int ntiles;         // td0 * td1 * td2 (the pseudo-tile "outside" is index ntiles)
  int max_chunks;
};

struct BinOutF {
  int* count;  // [ntiles + 1] (zeroed before a binning launch)
  int* ptile;  // [n]
  int* pslot;  // [n]
  int* tflag;  // [ntiles] (zeroed with count)
  FTiles tl;
};

// Arguments of k_fused that only rare paths use -- the re-binning launches'
// outputs, the escape path, impulses, tiles appended during the launch, the
// error flags, the once-a-chunk box publishing -- read through one pointer
// where they are used.  As kernel arguments they made ~150 dwords against
// 102 SGPRs, and the compiler kept 89 SGPRs spilled to VGPR lanes (348
// v_readlane restores in the code); now 38 (69).  k_fused's time did not
// move (5 interleaved rounds: 16.07 against 16.11 us steady), the same
// change to k_grid_f did (its slab-free form below).  One per (bins parity,
// escape flag) in device memory (mpm.hip sync_rare).
struct FusedRare {
  BinOutF bo;          // re-binning outputs (bins parity c ^ 1)
  float4* gacc;        // escape accumulator
  int* esc;            // escape flag this launch raises
  int* drift;          // slab: a particle past the margin (unused outside slabs)
  int* nonfin;         // non-finite state word
  const void* bct;     // const BcTable* (impulses)
  int* tflag;          // Touch members of add_lower_tiles (bins parity c)
  int* touched;
  int* nchunk;
  int4* chunk;
  int2* rcov;
  int* tbox;           // Touch's per-chunk box publishing (once a chunk: a scalar load, not a live SGPR)
  const int* tpos;
  int* rbox;
  // ---- the folded grid update (FOLD launches, below; null / unused otherwise) ----
  // Launch r of a step call (phase r mod 12) writes its chunk windows to the
  // slot buffer r mod 2, its tile boxes to tbox buffer r mod 2, its escapes to
  // gacc buffer r mod 3 and raises escape flag r mod 12.  The previous
  // launch's outputs are what a FOLD launch's staging reads:
  const float4* slots_prev;  // chunk windows of launch r - 1
  const int* tbox_prev;      // tile boxes of launch r - 1
  const float4* gacc_prev;   // escapes of launch r - 1 (read when *esc_prev)
  const int* esc_prev;       // escape flag of launch r - 1
  // launch r's housekeeping at its end: the escapes of launch r - 2 (read by
  // launch r - 1, written next by launch r + 1) are zeroed when *esc_old, and
  // flag r - 3 (read by launches r - 2 and r - 1) is cleared
  const int* esc_old;
  float4* gacc_old;
  int* esc_clr;
  float grav[3];  // gravity (f32): a FOLD launch forms dt * gravity as the host's grid_step does
  unsigned* esc_count;  // particle scatters that escaped their chunk window, summed (gsmpm_mpm_escapes)
  float4* esc_nodes;    // FOLD: [np][27] the stencil node values of a particle outside its chunk's window
  unsigned* vmax;       // G2P-only launches (a step call's last): max |v| component over the particles, as
                        // f32 bits (atomicMax), for the next call's re-binning count (mpm.hip choose_rebins)
};

// ---------------------------------------------------------------- the fold --
// FOLD launches (MODE bit 4) take the grid update of the previous substep
// into their own G2P staging instead of reading the dense v_out that a
// k_grid_f launch would have written: every node of the chunk's stencil box
// is summed from the chunk windows that cover it (the previous P2G's slots,
// in k_grid_f's fixed order: the node's owner tile's window first, then the
// covering neighbours by k_grid_f's e order, the second and further chunks
// after, the escape accumulator last), then normalised, gravity and the BC
// list applied (node_update, utils.py:177-183 + solver.py:41-46).  The staged
// value is bit-identical to k_grid_f's, so a step runs one launch per substep
// (k_grid_f only after a re-binning, whose next launch reads chunk windows of
// the old bins).  A node lies in up to 8 chunk windows (3.5 on average), so
// the slot bytes a launch reads grow by that factor over k_grid_f's; they come
// from L2 / MALL, written by the launch before.
constexpr int kFT[3] = {kFT0, kFT1, kFT2};
#ifndef GSMPM_FOLD_BATCH
#define GSMPM_FOLD_BATCH 1
#endif
constexpr int kFoldB = GSMPM_FOLD_BATCH;  // nodes a lane stages at once (their loads in flight together)
// per axis: window coordinate w (node o + w of tile t's window, o = t T - 1) ->
// the node's owner tile offset d in {-1, 0, 1} and k_grid_f's section sec of
// its owner-local coordinate l = w - 1 - d T (sec -1: l < 3, +1: l = T - 1)
__device__ __forceinline__ void fold_axis(int w, int T, int& d, int& sec) {
  d = w == 0 ? -1 : (w <= T ? 0 : 1);
  const int l = w - 1 - d * T;
  sec = l < 3 ? -1 : (l == T - 1 ? 1 : 0);
}
// (global address space: the loads may move across the staging's LDS stores)
__device__ __forceinline__ float4 ld_slot4(const float4* __restrict__ slots, int off) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef const f4v __attribute__((address_space(1)))* gf4_p;
  const f4v r = *(gf4_p)((const char*)slots + (unsigned)off * 16u);
  return make_float4(r.x, r.y, r.z, r.w);
}
__device__ __forceinline__ void add4f(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}
// The summed window value of one node from per-neighbour tables: covering
// tile e of the node is t + a_e (a_e per axis = d + (bit e ? sec : 0)), its
// {first chunk, chunks, box} read through `tab(ci, c0, nc, bx)` for the
// 27-neighbour index ci of a_e, and the node's coordinate in that window is
// w - a_e T.  Loads of covers outside the window's box (nothing was scattered
// there) are not issued.  Order of the sum: k_grid_f's (node_reads,
// node_extra).  fold_prep computes the 8 covers' slot offsets, fold_load
// issues their loads, fold_acc sums them (+ further chunks): split so a
// caller can have several nodes' loads in flight at once.
struct FoldNode {
  int off[8];  // first chunk's slot offset of each cover (valid where on)
  int on;      // bit e: cover e exists and its box holds the node
  int extra;   // bit e: ... and that cover's tile has further chunks
};
// cover e of window node w: its 27-neighbour index and the node's offset in its window
__device__ __forceinline__ void fold_cover(const int (&w)[3], int e, int& ci, int (&wn)[3], bool& valid) {
  int d[3], sec[3];
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) fold_axis(w[ax], kFT[ax], d[ax], sec[ax]);
  const int b0 = e >> 2, b1 = (e >> 1) & 1, b2 = e & 1;
  const int a0 = d[0] + (b0 ? sec[0] : 0), a1 = d[1] + (b1 ? sec[1] : 0), a2 = d[2] + (b2 ? sec[2] : 0);
  ci = (a0 + 1) * 9 + (a1 + 1) * 3 + (a2 + 1);
  wn[0] = w[0] - a0 * kFT0;
  wn[1] = w[1] - a1 * kFT1;
  wn[2] = w[2] - a2 * kFT2;
  valid = ((!b0) | (sec[0] != 0)) & ((!b1) | (sec[1] != 0)) & ((!b2) | (sec[2] != 0));
}
__device__ __forceinline__ bool in_box(const int (&wn)[3], int q) {
  return (wn[0] >= (q & 15)) & (wn[1] >= ((q >> 4) & 15)) & (wn[2] >= ((q >> 8) & 15)) & (wn[0] <= ((q >> 12) & 15)) &
         (wn[1] <= ((q >> 16) & 15)) & (wn[2] <= ((q >> 20) & 15));
}
template <typename Tab>
__device__ __forceinline__ void fold_prep(const int (&w)[3], Tab tab, FoldNode& f) {
  f.on = 0;
  f.extra = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    int ci, wn[3];
    bool valid;
    fold_cover(w, e, ci, wn, valid);
    int c0, nc, q;
    tab(ci, c0, nc, q);
    const bool on = valid & (nc > 0) & in_box(wn, q);
    f.on |= on ? (1 << e) : 0;
    f.extra |= (on & (nc > 1)) ? (1 << e) : 0;
    f.off[e] = c0 * kFWin + slot_loc(wn[0], wn[1], wn[2]);
  }
}
__device__ __forceinline__ void fold_load(const float4* __restrict__ slots, const FoldNode& f, float4 (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = ((f.on >> e) & 1) ? ld_slot4(slots, f.off[e]) : make_float4(0.f, 0.f, 0.f, 0.f);
}
// the sum: the first chunks in e order, then (rare: tiles of > 256 particles)
// the second chunks in e order and the third and later ones, their offsets
// recomputed from the tables (not kept live across the loads)
template <typename Tab>
__device__ __forceinline__ float4 fold_acc(const float4* __restrict__ slots, const int (&w)[3], Tab tab,
                                           const FoldNode& f, const float4 (&v)[8]) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int e = 0; e < 8; ++e) add4f(a, v[e]);
  if (f.extra) {
    int c0s[8], ncs[8], locs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int ci, wn[3];
      bool valid;
      fold_cover(w, e, ci, wn, valid);
      int q;
      tab(ci, c0s[e], ncs[e], q);
      locs[e] = slot_loc(wn[0], wn[1], wn[2]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float4 u = ((f.extra >> e) & 1) ? ld_slot4(slots, (c0s[e] + 1) * kFWin + locs[e])
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
      add4f(a, u);
    }
    // (an unrolled scan, not a ctz loop: a dynamic index would put the arrays in scratch)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if ((f.extra >> e) & 1)
        for (int c = c0s[e] + 2; c < c0s[e] + ncs[e]; ++c) add4f(a, ld_slot4(slots, c * kFWin + locs[e]));
  }
  return a;
}
template <typename Tab>
__device__ __forceinline__ float4 fold_sum(const float4* __restrict__ slots, const int (&w)[3], Tab tab) {
  FoldNode f;
  fold_prep(w, tab, f);
  float4 v[8];
  fold_load(slots, f, v);
  return fold_acc(slots, w, tab, f, v);
}

// The slow path: the updated velocity of any grid node (i, j, k) from the
// previous P2G's windows, through the tile tables of the node's owner tile
// (a particle of a FOLD launch that left its chunk's window, or one binned
// outside the grid).  0 outside the grid.
__device__ __forceinline__ float4 fold_node(int i, int j, int k, const GridDims& g, const FTiles& tl, const ChunkIn& ck,
                                            const FusedRare* __restrict__ rare, const GridStep& gs,
                                            const BcTable* __restrict__ bct, bool esc) {
  const int ng = g.ng;
  if ((unsigned)i >= (unsigned)ng || (unsigned)j >= (unsigned)ng || (unsigned)k >= (unsigned)ng)
    return make_float4(0.f, 0.f, 0.f, 0.f);
  const int ti = i / kFT0, tj = j / kFT1, tk = k / kFT2;
  // window coordinates of the node in its owner tile's window (owner offset d = 0)
  const int w[3] = {i - ti * kFT0 + 1, j - tj * kFT1 + 1, k - tk * kFT2 + 1};
  float4 a = fold_sum(rare->slots_prev, w, [&](int ci, int& c0, int& nc, int& q) {
    const int x = ti + ci / 9 - 1, y = tj + (ci / 3) % 3 - 1, z = tk + ci % 3 - 1;
    c0 = 0;
    nc = 0;
    q = 0;
    if ((unsigned)x < (unsigned)tl.td0 && (unsigned)y < (unsigned)tl.td1 && (unsigned)z < (unsigned)tl.td2) {
      const int u = (x * tl.td1 + y) * tl.td2 + z;
      c0 = ck.cbase[u];
      nc = (ck.count[u] + kChunk - 1) / kChunk;
      q = rare->tbox_prev[u];
    }
  });
  if (esc) add4f(a, rare->gacc_prev[((size_t)i * ng + j) * ng + k]);
  return node_update(a, i, j, k, g, gs, bct);
}

__device__ __forceinline__ void ftile_decode(const FTiles& tl, int t, int& tx, int& ty, int& tz) {
  tz = t % tl.td2;
  ty = (t / tl.td2) % tl.td1;
  tx = t / (tl.td1 * tl.td2);
}

// tile of a particle's base cell (utils.py:95 truncation), `ntiles` outside the grid
__device__ __forceinline__ int ftile_of(const float (&x)[3], const GridDims& g, const FTiles& tl, int (&tc)[3]) {
  bool ok = true;
  int b[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float gp = x[d] * g.inv_dx - 0.5f;
    ok = ok && (gp >= 0.0f) && (gp < (float)g.ng);  // false for NaN
    b[d] = ok ? (int)gp : 0;
  }
  tc[0] = b[0] / kFT0;
  tc[1] = b[1] / kFT1;
  tc[2] = b[2] / kFT2;
  return ok ? (tc[0] * tl.td1 + tc[1]) * tl.td2 + tc[2] : tl.ntiles;
}

// Touched tiles.  At binning time a tile's particles have their base cell in
// the tile, so their stencils reach the tiles t + {0, 1}^3: the first
// reservation in t flags those (idempotent plain stores).  A particle that
// later moves below its tile (base = tile origin - 1 on some axis) also
// reaches the lower neighbours; k_fused adds those to the touched list when
// it first sees such a particle in a chunk (add_lower_tiles).
__device__ __noinline__ void mark8(int* __restrict__ tflag, int t, int td0, int td1, int td2) {
  const int tz = t % td2, ty = (t / td2) % td1, tx = t / (td1 * td2);
  for (int a = 0; a <= 1; ++a)
    for (int b = 0; b <= 1; ++b)
      for (int c = 0; c <= 1; ++c)
        if (tx + a < td0 && ty + b < td1 && tz + c < td2) tflag[((tx + a) * td1 + ty + b) * td2 + tz + c] = 1;
}
__device__ __forceinline__ int reserve_f(const BinOutF& bo, int t, int c) {
  const int old = atomicAdd(&bo.count[t], c);
  if (old == 0 && t < bo.tl.ntiles) mark8(bo.tflag, t, bo.tl.td0, bo.tl.td1, bo.tl.td2);
  return old;
}

// The touched list of the bins a k_fused launch reads (the grid update that
// follows walks it) and the chunk records, whose .w holds the lower-neighbour
// axes already added for the chunk.
struct Touch {
  int* tflag;
  int* touched;
  int* nchunk;  // [1] = touched count
  int4* chunk;
  int* cbox;    // [max_chunks] stencil box of the chunk's last P2G (packed, window coordinates)
  int* tbox;    // [ntiles] the same per tile (the full window when the tile has several chunks)
  unsigned char* perm;  // [max_chunks][256] lane -> particle of the chunk (lane balance, below); null: off
  int2* rcov;           // cover records per touched position (ChunkIn): an appended tile's gets the "none" flag
  const int* tpos;      // [ntiles] touched position of each tile (-1: none); null: no box publishing
  int* rbox;            // [ntiles][kRecStride] the neighbours' stencil boxes of this substep, per touched position
};

// Lane balance.  A wave's LDS accesses to the chunk window (G2P's ds_read_b128
// of float4 nodes, P2G's 64-bit atomics into channel planes) are serviced in
// lane groups of 16 whose banks follow the node index mod 16 -- and with the
// same stencil offset added by every lane, a group is conflict-free exactly
// when its 16 particles' base nodes are distinct mod 16.  Every P2G records,
// per chunk, the lane assignment that puts a particle whose base node has
// residue r on a lane L with L mod 16 = r wherever the residue counts allow
// (the leftovers fill the remaining lanes in order); the next launch on the
// same bins (the particles moved < 1 cell) runs its lanes through it.  Both
// b128 and b64 lane groups hold 16 lanes of distinct L mod 16.
__device__ __forceinline__ int balanced_lane(const int* __restrict__ rcnt, int cnt, int r, int rank) {
  const int Lr = (cnt - r + 15) >> 4;  // lanes of residue r in [0, cnt)
  if (rank < Lr) return rank * 16 + r;
  int o = rank - Lr;
  for (int q = 0; q < r; ++q) o += max(0, rcnt[q] - ((cnt - q + 15) >> 4));
  int acc = 0;
  for (int q = 0; q < 16; ++q) {
    const int Lq = (cnt - q + 15) >> 4, d = max(0, Lq - rcnt[q]);
    if (o < acc + d) return (rcnt[q] + (o - acc)) * 16 + q;
    acc += d;
  }
  return rank * 16 + r;  // unreachable: overflow == deficit
}

// Stencil boxes: lo/hi window coordinates (0..11) per axis in 4-bit fields,
// lo0 | lo1 << 4 | lo2 << 8 | hi0 << 12 | hi1 << 16 | hi2 << 20.  The P2G of
// a chunk writes only the nodes inside its box, the next G2P of the chunk
// stages only those (the particles have not moved in between), and the grid
// update reads a tile's windows only inside its box.
constexpr int kFullBox = 0 | (0 << 4) | (0 << 8) | ((kFW0 - 1) << 12) | ((kFW1 - 1) << 16) | ((kFW2 - 1) << 20);
__device__ __forceinline__ void box_unpack(int b, int (&lo)[3], int (&hi)[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    lo[d] = (b >> (4 * d)) & 15;
    hi[d] = (b >> (12 + 4 * d)) & 15;
  }
}

// Lanes 0..26: add the tiles t + a, a_d in {-1 if d in lo, 0, 1}, with some
// a_d = -1, that are not yet flagged (one append per tile: the flag CAS).
__device__ __forceinline__ void add_lower_tiles(const Touch& tc, const FTiles& tl, int tx, int ty, int tz, int lo) {
  const int e = threadIdx.x;
  if (e < 27) {
    const int a = e / 9 - 1, b = (e / 3) % 3 - 1, c = e % 3 - 1;
    const bool need = (a < 0 || b < 0 || c < 0) && (a >= 0 || (lo & 1)) && (b >= 0 || (lo & 2)) && (c >= 0 || (lo & 4));
    const int x = tx + a, y = ty + b, z = tz + c;
    if (need && (unsigned)x < (unsigned)tl.td0 && (unsigned)y < (unsigned)tl.td1 && (unsigned)z < (unsigned)tl.td2) {
      const int t = (x * tl.td1 + y) * tl.td2 + z;
      if (atomicCAS(&tc.tflag[t], 0, 1) == 0) {
        const int pos = atomicAdd(&tc.nchunk[1], 1);
        tc.touched[pos] = t;
        // no cover record (its neighbours publish no boxes for it): k_grid_f reads the tile tables
        if (tc.rcov) tc.rcov[(size_t)pos * kRecStride + 27] = make_int2(1, 0);
      }
    }
  }
}

// base cell of a particle as bspline() computes it
__device__ __forceinline__ void base_of(const float (&x)[3], float inv_dx, int (&b)[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) b[d] = (int)(x[d] * inv_dx - 0.5f);
}

// Escapes and the grid update.  A particle that scatters through the dense
// accumulator (p2g_global: it left its chunk's window, or its chunk lies
// outside the grid) adds the tiles owning its in-grid stencil nodes to the
// touched list, as add_lower_tiles does for a new lower neighbour, so the
// next k_grid_f -- which adds the accumulator to the nodes it owns and zeroes
// it -- finds every node an escape wrote among the touched tiles.  Round 5
// swept every tile of the grid after any escape (4,864 tiles at 128^3 against
// ~900 touched); GSMPM_ESC_SWEEP=1 restores that (A/B).
#ifndef GSMPM_ESC_SWEEP
#define GSMPM_ESC_SWEEP 0
#endif
constexpr bool kEscSweepAll = GSMPM_ESC_SWEEP != 0;
__device__ __forceinline__ void mark_escape_tiles(int* __restrict__ tflag, int* __restrict__ touched,
                                               int* __restrict__ ntouch, int2* __restrict__ rcov, const FTiles& tl,
                                               int ng, int b0, int b1, int b2) {
  const int lo0 = max(b0, 0), lo1 = max(b1, 0), lo2 = max(b2, 0);
  const int hi0 = min(b0 + 2, ng - 1), hi1 = min(b1 + 2, ng - 1), hi2 = min(b2 + 2, ng - 1);
  if (lo0 > hi0 || lo1 > hi1 || lo2 > hi2) return;  // no stencil node in the grid
  for (int a = lo0 / kFT0; a <= hi0 / kFT0; ++a)
    for (int c = lo1 / kFT1; c <= hi1 / kFT1; ++c)
      for (int e = lo2 / kFT2; e <= hi2 / kFT2; ++e) {
        const int t = (a * tl.td1 + c) * tl.td2 + e;
        if (__hip_atomic_load(&tflag[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
            atomicCAS(&tflag[t], 0, 1) == 0) {
          const int pos = atomicAdd(ntouch, 1);
          touched[pos] = t;
          if (rcov) rcov[(size_t)pos * kRecStride + 27] = make_int2(1, 0);  // no cover record: the tile tables
        }
      }
}
// stencil inside the chunk window whose first node is o
__device__ __forceinline__ bool in_window(const int (&b)[3], int o0, int o1, int o2) {
  return (unsigned)(b[0] - o0) <= (unsigned)(kFW0 - 3) && (unsigned)(b[1] - o1) <= (unsigned)(kFW1 - 3) &&
         (unsigned)(b[2] - o2) <= (unsigned)(kFW2 - 3);
}
// the per-phase pipeline's in-grid test (tile_of): base cell inside [0, ng)^3
__device__ __forceinline__ bool in_grid(const float (&x)[3], const GridDims& g) {
  bool ok = true;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float gp = x[d] * g.inv_dx - 0.5f;
    ok = ok && (gp >= 0.0f) && (gp < (float)g.ng);
  }
  return ok;
}

// MODE bit 1: G2P of the previous grid update; bit 2: P2G of this substep.
// `bin` (uniform): re-bin the particles by their new x into `bo`.
// Particle storage is in bin order (permuted at every binning), so chunk w's
// particles are storage rows [first, first + cnt).
#ifndef GSMPM_STORE_VC
#define GSMPM_STORE_VC 0  // 1: every G2P stores v and C (A/B)
#endif
// GSMPM_ZERO_BOX=1: the P2G half zeroes only its chunk's store box of the LDS
// window (the nodes its stencils reach: ~57 % of the 1,584 on the lego
// frame), once the box is known, with one more workgroup barrier, instead
// of the whole window before it.  Measured and rejected (round 4, 2 A/B
// rounds on the lego bench, profiles/r04/ab_libs_r04e.txt): sim 3.120 / 3.129
// against 3.115 / 3.100 ms/frame, k_fused 17.0 against 16.9 us -- the zeroing
// is hidden under the particle loads it overlaps; the barrier is not
#ifndef GSMPM_ZERO_BOX
#define GSMPM_ZERO_BOX 0
#endif
constexpr bool kZeroBox = GSMPM_ZERO_BOX != 0;
// GSMPM_ATOMIC_GRID=1: the P2G half adds its window box into the dense
// accumulator gacc with global float atomics (one lane per node channel)
// instead of storing it to the chunk's slot, and k_grid_f reads one node of
// gacc (and zeroes it) instead of summing <= 8 covering slots through the
// 27-tile cover table.  The cross-chunk sum becomes order-dependent f32 (as
// the reference's Taichi atomics are); within a chunk it stays exact (A/B)
#ifndef GSMPM_ATOMIC_GRID
#define GSMPM_ATOMIC_GRID 0
#endif
constexpr bool kAtomicGrid = GSMPM_ATOMIC_GRID != 0;
// GSMPM_SIM_PRIO=n (A/B): the simulator's waves raise their issue priority
// (s_setprio n, 0..3) so that a SIMD's arbiter serves them before the waves of
// the render of the previous frame, which runs on a second stream beside them
// (the frame costs sim + ~0.25 ms of that render's interference, §6)
#ifndef GSMPM_SIM_PRIO
#define GSMPM_SIM_PRIO 0
#endif
constexpr int kSimPrio = GSMPM_SIM_PRIO;
__device__ __forceinline__ void sim_prio() {
  if constexpr (kSimPrio > 0) __builtin_amdgcn_s_setprio(kSimPrio);
}
#ifndef GSMPM_DPP_REDUCE
#define GSMPM_DPP_REDUCE 1
#endif
// GSMPM_G2P_B128 (A/B, default 1): G2P's 27 LDS gathers as ds_read_b128
#ifndef GSMPM_G2P_B128
#define GSMPM_G2P_B128 1
#endif
constexpr bool kG2pB128 = GSMPM_G2P_B128 != 0;
#ifndef GSMPM_BIN_AGG
#define GSMPM_BIN_AGG 1
#endif
constexpr bool kBinAgg = GSMPM_BIN_AGG != 0;
// bin: 1 = re-bin the particles by their new x into rare->bo; 2 = zero
// rare->bo's counts and flags for the next launch's re-binning (at the end)
template <int MAT, int MODE>
__global__ __launch_bounds__(256, 3) void k_fused(Particles ps, GridDims g, FTiles tl, ChunkIn ck, Touch tc, int bin,
                                               int use_box, const float4* __restrict__ gvel, uint32_t mask, float dt,
                                               MatConsts mc, float4* __restrict__ slots, int xlo, int xhi,
                                               const FusedRare* __restrict__ rare, uint32_t mask_prev) {
  constexpr bool G2P = (MODE & 1) != 0, P2G = (MODE & 2) != 0;
  constexpr bool FOLD = G2P && (MODE & 4) != 0;  // the previous substep's grid update staged from its chunk windows
  __shared__ int s_fc0[27], s_fnc[27], s_fbx[27];  // FOLD: the 27 neighbour tiles' tables
  // FOLD: particles outside their chunk's window (escapes; rare): their stencil
  // nodes are evaluated by the whole workgroup into the upper half of s_acc
  // (free while G2P runs: the v window uses the lower half), kEscMax at a time
  constexpr int kEscMax = kFWin / 27;
  __shared__ int s_nesc;
  __shared__ int s_eb[3][kEscMax];
  // FOLD: the previous substep's grid step, and whether its P2G had escapes (uniform)
  GridStep fgs{};
  bool fesc = false;
  if constexpr (FOLD) {
    fgs.dt = dt;
    fgs.dgx = dt * rare->grav[0];
    fgs.dgy = dt * rare->grav[1];
    fgs.dgz = dt * rare->grav[2];
    fgs.mask = mask_prev;
    fgs.keep = 0;
    fesc = __builtin_amdgcn_readfirstlane(*rare->esc_prev) != 0;
  }
  // channel-planar u64 accumulators; the G2P v window aliases them (it is
  // consumed before the accumulators are zeroed)
  __shared__ unsigned long long s_acc[4 * kFWin];
  __shared__ float s_max[4];
  __shared__ int s_mxy[4], s_mz[4];
  __shared__ int s_cnt[27], s_base[27];
  __shared__ int s_rcnt[16];
  float4* s_win = reinterpret_cast<float4*>(s_acc);
  const int ng = g.ng;
  constexpr int SK = (MODE & 3) == 3 ? 0 : 1;  // diagnostics slot (k_p2g's / k_g2p's in the per-phase pipeline)
  sim_prio();
  stamp(SK, 0);
  // the first chunk's record, box and lane order are requested with the chunk
  // count (clamped: a workgroup past the last chunk discards them), which
  // takes dependent round trips off every workgroup's chain (the same for
  // every further chunk: its record, box and lane order are requested while
  // the chunk before it is processed).  The empty asm takes the pointers
  // into SGPRs in the first argument batch and the loads go through the
  // global address space as vector loads, so all four leave together: as
  // plain scalar loads the compiler serialised them -- box, then count, then
  // record, three memory round trips behind each other at the kernel start
  // (one shared lgkmcnt, argument reloads between them)
  // (all four unconditional, straight-line: an unused lane order reads
  // cbox[0] instead, selected away below)
  const int w0 = min((int)blockIdx.x, tl.max_chunks - 1);
  const bool perm0 = use_box && tc.perm;
  const int* nch_p = ck.nchunk;
  const int4* chk_p = ck.chunk;
  const int* cbx_p = tc.cbox;
  const unsigned char* prm_p = perm0 ? tc.perm : reinterpret_cast<const unsigned char*>(tc.cbox);
  asm volatile("" : "+s"(nch_p), "+s"(chk_p), "+s"(cbx_p), "+s"(prm_p));
  typedef const int __attribute__((address_space(1)))* gint_p;
  typedef const unsigned char __attribute__((address_space(1)))* guc_p;
  const gint_p c4 = (gint_p)chk_p + 4 * (size_t)w0;
  const int r0 = c4[0], r1 = c4[1], r2 = c4[2], r3 = c4[3];
  const int bx0 = ((gint_p)cbx_p)[w0];
  const int qv0 = ((guc_p)prm_p)[perm0 ? (size_t)w0 * 256 + threadIdx.x : 0];
  const int nch = *(gint_p)nch_p;
  int4 cr_n = make_int4(r0, r1, r2, r3);
  int box_n = use_box ? bx0 : kFullBox;
  int q_n = perm0 ? qv0 : (int)threadIdx.x;
  for (int w = blockIdx.x; w < nch; w += gridDim.x) {
    const int4 cr = cr_n;
    const int cbox = box_n, q_lane = q_n;
    if (w + (int)gridDim.x < nch) {  // workgroup-uniform; chunk w + grid is only ever touched by this workgroup
      const int wn = w + gridDim.x;
      cr_n = ck.chunk[wn];
      box_n = use_box ? tc.cbox[wn] : kFullBox;
      q_n = (use_box && tc.perm) ? (int)tc.perm[(size_t)wn * 256 + threadIdx.x] : (int)threadIdx.x;
    }
    const int t = cr.x, first = cr.y, cnt = cr.z;
    const int k = threadIdx.x;
    const bool outside = t == tl.ntiles;  // workgroup-uniform
    int tx = 0, ty = 0, tz = 0;
    if (!outside) ftile_decode(tl, t, tx, ty, tz);
    const int o0 = tx * kFT0 - 1, o1 = ty * kFT1 - 1, o2 = tz * kFT2 - 1;  // first window node
    // lane e < 27: the touched position of tile T = t - (a, b, c), whose cover
    // record takes this chunk's stencil box as its neighbour e (published after
    // the P2G below); requested now, used at the end
    int tpos_e = -1;
    const int* __restrict__ tposp = rare->tpos;
    if (tposp && !outside && k < 27) {
      const int x0 = tx - (k / 9 - 1), y0 = ty - ((k / 3) % 3 - 1), z0 = tz - (k % 3 - 1);
      if ((unsigned)x0 < (unsigned)tl.td0 && (unsigned)y0 < (unsigned)tl.td1 && (unsigned)z0 < (unsigned)tl.td2)
        tpos_e = tposp[(x0 * tl.td1 + y0) * tl.td2 + z0];
    }
    int p = -1;
    float x[3] = {0.f, 0.f, 0.f}, v[3] = {0.f, 0.f, 0.f}, C[3][3], F[3][3], m = 0.f;
    // this lane's particle: the lane balance of the last P2G on these bins (use_box), else in order
    const int q = k >= cnt ? k : q_lane;
    // particle loads first: their round trips overlap the window staging
    if (k < cnt) {
      p = first + q;
#pragma unroll
      for (int d = 0; d < 3; ++d) x[d] = ps.ld(PX + d, p);
      if (G2P || MAT != 0) {
#pragma unroll
        for (int i = 0; i < 9; ++i) F[i / 3][i % 3] = ps.ld(PF + i, p);
      }
      if (P2G) m = ps.ld(PMASS, p);
      if (!G2P) {
#pragma unroll
        for (int d = 0; d < 3; ++d) v[d] = ps.ld(PV + d, p);
#pragma unroll
        for (int i = 0; i < 9; ++i) C[i / 3][i % 3] = ps.ld(PC + i, p);
      }
    }
    int eslot = -1;  // FOLD: this lane's escape slot (its stencil nodes at s_win[kFWin + 27 eslot ...])
    if constexpr (G2P) {
      if (FOLD && !outside) {
        // the 27 neighbour tiles' first chunk, chunk count and stencil box of the previous P2G (lanes 0..26)
        if (k < 27) {
          const int x0 = tx + k / 9 - 1, y0 = ty + (k / 3) % 3 - 1, z0 = tz + k % 3 - 1;
          int c0 = 0, nc = 0, bx = 0;
          if ((unsigned)x0 < (unsigned)tl.td0 && (unsigned)y0 < (unsigned)tl.td1 && (unsigned)z0 < (unsigned)tl.td2) {
            const int u = (x0 * tl.td1 + y0) * tl.td2 + z0;
            c0 = ck.cbase[u];
            nc = (ck.count[u] + kChunk - 1) / kChunk;
            bx = rare->tbox_prev[u];
          }
          s_fc0[k] = c0;
          s_fnc[k] = nc;
          s_fbx[k] = bx;
        }
        if (k == 0) s_nesc = 0;
        __syncthreads();
        // a lane whose particle left the window takes an escape slot (its base in s_eb)
        if (k < cnt) {
          int bq[3];
          base_of(x, g.inv_dx, bq);
          if (!(in_grid(x, g) && in_window(bq, o0, o1, o2))) {
            eslot = atomicAdd(&s_nesc, 1);
            if (eslot < kEscMax) {
              s_eb[0][eslot] = bq[0];
              s_eb[1][eslot] = bq[1];
              s_eb[2][eslot] = bq[2];
            }
          }
        }
        int lo[3], hi[3];
        box_unpack(cbox, lo, hi);
        const int n1 = hi[1] - lo[1] + 1, n2 = hi[2] - lo[2] + 1, n12 = n1 * n2;
        const int nvol = (hi[0] - lo[0] + 1) * n12;
        const float r12 = 1.0f / (float)n12, r2 = 1.0f / (float)n2;
        const float4* __restrict__ sp = rare->slots_prev;
        const BcTable* __restrict__ fbct = static_cast<const BcTable*>(rare->bct);
        auto tab = [&](int ci, int& c0, int& nc, int& q) {
          c0 = s_fc0[ci];
          nc = s_fnc[ci];
          q = s_fbx[ci];
        };
        // kFoldB nodes a lane at a time: all their cover loads in flight together
        for (int q0 = k; q0 < nvol; q0 += 256 * kFoldB) {
          FoldNode fn[kFoldB];
          int w3[kFoldB][3];
          bool gin[kFoldB], live[kFoldB];
#pragma unroll
          for (int u = 0; u < kFoldB; ++u) {
            const int qn = min(q0 + u * 256, nvol - 1);
            live[u] = q0 + u * 256 < nvol;
            const int a = (int)(((float)qn + 0.5f) * r12), rem = qn - a * n12;
            const int b = (int)(((float)rem + 0.5f) * r2), c = rem - b * n2;
            w3[u][0] = lo[0] + a;
            w3[u][1] = lo[1] + b;
            w3[u][2] = lo[2] + c;
            const int ix = o0 + w3[u][0], iy = o1 + w3[u][1], iz = o2 + w3[u][2];
            gin[u] = live[u] && (unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng;
            fold_prep(w3[u], tab, fn[u]);
            if (!gin[u]) fn[u].on = 0;
          }
          float4 vv[kFoldB][8];
#pragma unroll
          for (int u = 0; u < kFoldB; ++u) fold_load(sp, fn[u], vv[u]);
#pragma unroll
          for (int u = 0; u < kFoldB; ++u) {
            const int ix = o0 + w3[u][0], iy = o1 + w3[u][1], iz = o2 + w3[u][2];
            float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gin[u]) {
              float4 sum = fold_acc(sp, w3[u], tab, fn[u], vv[u]);
              if (fesc) add4f(sum, rare->gacc_prev[((size_t)ix * ng + iy) * ng + iz]);
              val = node_update(sum, ix, iy, iz, g, fgs, fbct);
            }
            if (live[u]) s_win[(w3[u][0] * kFW1 + w3[u][1]) * kFW2 + w3[u][2]] = val;
          }
        }
        // the escaped particles' stencil nodes, one node a lane (workgroup-uniform skip when none)
        __syncthreads();
        const int ne = min(s_nesc, kEscMax);
        for (int t = k; t < ne * 27; t += 256) {
          const int sl = t / 27, qn = t - sl * 27;
          s_win[kFWin + t] = fold_node(s_eb[0][sl] + qn / 9, s_eb[1][sl] + (qn / 3) % 3, s_eb[2][sl] + qn % 3, g, tl,
                                       ck, rare, fgs, fbct, fesc);
        }
      } else if (!outside) {
        // the chunk's stencil box from its last P2G (particles unmoved since), else the whole window
        int lo[3], hi[3];
        box_unpack(cbox, lo, hi);
        const int n1 = hi[1] - lo[1] + 1, n2 = hi[2] - lo[2] + 1, n12 = n1 * n2;
        const int nvol = (hi[0] - lo[0] + 1) * n12;
        const float r12 = 1.0f / (float)n12, r2 = 1.0f / (float)n2;  // exact floor for q < 2^11
        constexpr int kStageU = (kFWin + 255) / 256;  // window nodes per lane, at most
        // all loads first, the out-of-grid zeroing as a select afterwards: a
        // zeroing branch right after each load made the compiler wait for
        // that load before issuing the next (the zeros and the in-flight load
        // share the registers), 7 round trips in a row instead of one
        float4 gv[kStageU];
        int dst[kStageU];
        bool gin[kStageU];
#pragma unroll
        for (int u = 0; u < kStageU; ++u) {
          const int qn = min(k + u * 256, nvol - 1);
          const int a = (int)(((float)qn + 0.5f) * r12), rem = qn - a * n12;
          const int b = (int)(((float)rem + 0.5f) * r2), c = rem - b * n2;
          const int wa = lo[0] + a, wb = lo[1] + b, wc = lo[2] + c;
          dst[u] = (wa * kFW1 + wb) * kFW2 + wc;
          const int ix = o0 + wa, iy = o1 + wb, iz = o2 + wc;
          gin[u] = (unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng;
          gv[u] = gvel[gin[u] ? ((size_t)ix * ng + iy) * ng + iz : 0];
        }
#pragma unroll
        for (int u = 0; u < kStageU; ++u) {
          const float4 z = gv[u];
          const bool in = gin[u];
          const float4 val = make_float4(in ? z.x : 0.f, in ? z.y : 0.f, in ? z.z : 0.f, in ? z.w : 0.f);
          if (k + u * 256 < nvol) s_win[dst[u]] = val;
        }
      }
      if (k < 27) s_cnt[k] = 0;
      __syncthreads();
      if (w == (int)blockIdx.x) {
        stamp(SK, 2);
        stamp_val(SK, 5, cnt);
        stamp_val(SK, 6, GSMPM_HWREG(4));   // HW_ID
        stamp_val(SK, 7, GSMPM_HWREG(20));  // XCC_ID
      }
      int code = -1, lslot = 0, nt = -1;
      if (k < cnt) {
        int b[3];
        base_of(x, g.inv_dx, b);
        float gvd[3][3];
        const bool inwin = !outside && in_grid(x, g) && in_window(b, o0, o1, o2);
        const bool eslds = eslot >= 0 && eslot < kEscMax;  // nodes evaluated by the workgroup (LDS)
        if (FOLD && !inwin && !eslds) {
          // the outside chunk, or more escapes than LDS slots (rarer still): this
          // lane's 27 stencil nodes one at a time through the owner tiles' tables,
          // into its rows of esc_nodes (a rolled loop: no call, no stack)
          float4* en = rare->esc_nodes + (size_t)p * 27;
#pragma unroll 1
          for (int qn = 0; qn < 27; ++qn)
            en[qn] = fold_node(b[0] + qn / 9, b[1] + (qn / 3) % 3, b[2] + qn % 3, g, tl, ck, rare, fgs,
                               static_cast<const BcTable*>(rare->bct), fesc);
        }
        if (inwin) {
          g2p_gather<kG2pB128>(x, g,
                     [&](const int (&base)[3], int i, int j, int kk) {
                       const int q = ((base[0] - o0 + i) * kFW1 + (base[1] - o1 + j)) * kFW2 + (base[2] - o2 + kk);
                       return s_win[q];
                     },
                     v, C, gvd);
        } else {
          g2p_gather(x, g,
                     [&](const int (&base)[3], int i, int j, int kk) {
                       const int ix = base[0] + i, iy = base[1] + j, iz = base[2] + kk;
                       float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
                       if constexpr (FOLD) {
                         const int qn = i * 9 + j * 3 + kk;
                         r = eslds ? s_win[kFWin + eslot * 27 + qn] : rare->esc_nodes[(size_t)p * 27 + qn];
                       } else {
                         if ((unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng)
                           r = gvel[((size_t)ix * ng + iy) * ng + iz];
                       }
                       return r;
                     },
                     v, C, gvd);
        }
        float Fn[3][3];
        f_trial(gvd, F, dt, Fn);
        // v and C: stored by the last launch of a step only.  The P2G half
        // takes them from registers, and the next launch's G2P recomputes
        // both from the grid, so a G2P + P2G launch's copies are never read.
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          if (!P2G || GSMPM_STORE_VC) ps.st(PV + d, p, v[d]);
          x[d] = x[d] + dt * v[d];
          ps.st(PX + d, p, x[d]);
        }
        if (!finite3(x)) *rare->nonfin = 1;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
          if (!P2G || GSMPM_STORE_VC) ps.st(PC + i, p, C[i / 3][i % 3]);
          F[i / 3][i % 3] = Fn[i / 3][i % 3];
        }
        // F_trial is stored here unless the return map below replaces it
        if (!P2G || MAT == 0 || MAT == 4) {
#pragma unroll
          for (int i = 0; i < 9; ++i) ps.st(PF + i, p, F[i / 3][i % 3]);
        }
        if (bin == 1) {
          int tc[3];
          nt = ftile_of(x, g, tl, tc);
          if (!outside && nt < tl.ntiles) {
            const int d0 = tc[0] - tx, d1 = tc[1] - ty, d2 = tc[2] - tz;
            if (abs(d0) <= 1 && abs(d1) <= 1 && abs(d2) <= 1) code = (d0 + 1) * 9 + (d1 + 1) * 3 + (d2 + 1);
          }
        }
      }
      if (bin == 1) {
        // the slot of the particle in its new tile's bin, reserved once per
        // (wave, neighbour tile): nearly every lane of a wave stays in the
        // chunk's own tile, and one LDS counter hit by 64 lanes serializes
        // them (2 cycles a lane, ~half of round 4's k_fused LDS bank-conflict
        // cycles); GSMPM_BIN_AGG=0: a lane-level atomic (A/B)
        if constexpr (kBinAgg) {
          unsigned long long pending = __ballot(code >= 0);
          while (pending) {  // wave-uniform: one trip per distinct neighbour tile of the wave
            const int lead = __ffsll(pending) - 1;
            const int lc = __builtin_amdgcn_readlane(code, lead);
            const unsigned long long mk = __ballot(code == lc);
            int base = 0;
            if ((k & 63) == lead) base = atomicAdd(&s_cnt[lc], __popcll(mk));
            base = __builtin_amdgcn_readlane(base, lead);
            if (code == lc)
              lslot = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mk >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mk, 0u));
            pending &= ~mk;
          }
        } else if (code >= 0) {
          lslot = atomicAdd(&s_cnt[code], 1);
        }
        __syncthreads();
        if (k < 27) {
          const int c = s_cnt[k];
          if (c > 0) {
            const int ntile = ((tx + k / 9 - 1) * tl.td1 + (ty + (k / 3) % 3 - 1)) * tl.td2 + (tz + k % 3 - 1);
            s_base[k] = reserve_f(rare->bo, ntile, c);
          }
        }
        __syncthreads();
        if (p >= 0) {
          const BinOutF bo = rare->bo;
          bo.ptile[p] = nt;
          bo.pslot[p] = code >= 0 ? s_base[code] + lslot : reserve_f(bo, nt, 1);
        }
      }
      if constexpr (!P2G) {  // the call's last launch: the particles' fastest velocity component
        float vm = 0.f;
        if (k < cnt) vm = fmaxf(fabsf(v[0]), fmaxf(fabsf(v[1]), fabsf(v[2])));
        if (!(vm <= 3.0e38f)) vm = 3.0e38f;  // NaN / Inf (flagged elsewhere): keep the bits ordered
        vm = wave_max_nonneg_dpp(vm);
        if ((k & 63) == 0 && vm > 0.f && rare->vmax) atomicMax(rare->vmax, __float_as_uint(vm));
      }
      __syncthreads();  // the window is consumed (and s_cnt / s_base read) before LDS is reused
      if (w == (int)blockIdx.x) stamp(SK, 3);
    }
    if constexpr (P2G) {
      if (!outside && !kZeroBox) {  // 16-byte stores: half the LDS write instructions of u64 ones
        uint4* z = reinterpret_cast<uint4*>(s_acc);
        for (int e = k; e < kFWin * 2; e += 256) z[e] = make_uint4(0u, 0u, 0u, 0u);
      }
      if (k < 16) s_rcnt[k] = 0;
      float nvt[3][3];
#pragma unroll
      for (int i = 0; i < 9; ++i) nvt[i / 3][i % 3] = 0.f;
      float bound = 0.f;
      if (k < cnt) {
        // ImpulseBC.apply (boundary_conditions.py:41-45); the kicked v lives in registers only
        if (mask) {
          const BcTable* __restrict__ bct = static_cast<const BcTable*>(rare->bct);
          const int ni = bct->n_imp;
          for (int b = 0; b < ni; ++b) {
            const Impulse& im = bct->imp[b];
            if (!((mask >> im.bit) & 1u)) continue;
            const bool in = fabsf(x[0] - im.c[0]) < im.s[0] && fabsf(x[1] - im.c[1]) < im.s[1] &&
                            fabsf(x[2] - im.c[2]) < im.s[2];
            if (in) {
#pragma unroll
              for (int d = 0; d < 3; ++d) v[d] = v[d] + im.f[d] / m * im.sdt;
            }
          }
        }
        // compute_stress_from_F_trial (utils.py:13-54)
        if constexpr (MAT != 0) {
          float tau[3][3];
          float yld = ps.ld(PYLD, p);
          const float mu = ps.ld(PMU, p), lam = ps.ld(PLAM, p);
          return_map_and_stress<MAT>(F, mu, lam, yld, dt, mc, tau);
          if constexpr (MAT == 1 || MAT == 2 || MAT == 3) {
#pragma unroll
            for (int i = 0; i < 9; ++i) ps.st(PF + i, p, F[i / 3][i % 3]);
          }
          if constexpr (MAT == 1) ps.st(PYLD, p, yld);
          const float nvol = -ps.ld(PVOL, p);
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) nvt[i][j] = nvol * tau[i][j];
        }
        // non-finite inputs of the scatter (a NaN / Inf would turn into finite
        // garbage through the fixed-point conversion, not propagate as the
        // reference's float atomics do): mass, velocity (impulse), stress, and
        // in a P2G-only launch the x and C it starts from
        {
          float chk = m + v[0] + v[1] + v[2];
          if constexpr (MAT != 0) {
#pragma unroll
            for (int i = 0; i < 9; ++i) chk += nvt[i / 3][i % 3];
          }
          if constexpr (!G2P) {
            chk += x[0] + x[1] + x[2];
#pragma unroll
            for (int i = 0; i < 9; ++i) chk += C[i / 3][i % 3];
          }
          if (!__builtin_isfinite(chk)) *rare->nonfin = 1;
        }
        float vm = 0.f, cm = 0.f, sm = 0.f;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          vm = fmaxf(vm, fabsf(v[r]));
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            cm = fmaxf(cm, fabsf(C[r][c]));
            sm = fmaxf(sm, fabsf(nvt[r][c]));
          }
        }
        bound = fmaxf(m, m * (vm + 4.5f * g.dx * cm) + dt * 4.5f * g.inv_dx * sm) * 1.01f;
      }
      if (outside) {
        // chunk of particles binned outside the grid: bounds-checked global path
        if (k < cnt) {
          p2g_global<MAT>(x, v, C, m, nvt, g, dt, rare->gacc);
          int bq[3];
          base_of(x, g.inv_dx, bq);
          if (!kEscSweepAll) mark_escape_tiles(rare->tflag, rare->touched, rare->nchunk + 1, rare->rcov, tl, ng, bq[0], bq[1], bq[2]);
        }
        if (k == 0 && cnt > 0) {
          *rare->esc = 1;
          atomicAdd(rare->esc_count, (unsigned)cnt);
        }
        // the next launch on these bins reads this chunk's lane order too: the
        // identity (round 4 left it unwritten, so a lane of the next G2P took a
        // stale row -- another chunk's particle, or one past the live rows)
        if (tc.perm && k < cnt) tc.perm[(size_t)w * 256 + k] = (unsigned char)q;
        __syncthreads();
        continue;  // workgroup-uniform
      }
      int b[3];
      base_of(x, g.inv_dx, b);
      const bool win = k < cnt && in_grid(x, g) && in_window(b, o0, o1, o2);
      // slab: a particle past the margin scatters where no window exchange reaches (slab.h)
      if (k < cnt && (b[0] < xlo || b[0] >= xhi)) *rare->drift = 1;
      // window coordinates covered by this particle's stencil, as per-axis bit masks
      int mxy = win ? (7 << (b[0] - o0)) | (7 << (16 + b[1] - o1)) : 0;
      int mz = win ? 7 << (b[2] - o2) : 0;
      // wave reductions by DPP (the bound is >= 0; a NaN bound -- non-finite
      // inputs, flagged above -- orders above every finite one as integer bits);
      // GSMPM_DPP_REDUCE=0 (A/B): shuffles (ds_bpermute_b32)
      if constexpr (GSMPM_DPP_REDUCE != 0) {
        bound = wave_max_nonneg_dpp(bound);
        mxy = wave_or_dpp(mxy);
        mz = wave_or_dpp(mz);
      } else {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          bound = fmaxf(bound, __shfl_xor(bound, o));
          mxy |= __shfl_xor(mxy, o);
          mz |= __shfl_xor(mz, o);
        }
      }
      if ((k & 63) == 0) {
        s_max[k >> 6] = bound;
        s_mxy[k >> 6] = mxy;
        s_mz[k >> 6] = mz;
      }
      __syncthreads();  // also orders the zeroing before the adds
      // lane balance for the next launch: this particle's rank among those of its base-node residue
      const int res = win ? (((b[0] - o0) * kFW1 + (b[1] - o1)) * kFW2 + (b[2] - o2)) & 15 : (q & 15);
      const int rrank = (tc.perm && k < cnt) ? atomicAdd(&s_rcnt[res], 1) : 0;
      const float bmax = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
      const int Mxy = s_mxy[0] | s_mxy[1] | s_mxy[2] | s_mxy[3], Mz = s_mz[0] | s_mz[1] | s_mz[2] | s_mz[3];
      const int Mx = Mxy & 0xffff, My = (unsigned)Mxy >> 16;
      // axes on which some stencil reaches below the tile (window coordinate 0)
      const int lo_all = (Mx & 1) | ((My & 1) << 1) | ((Mz & 1) << 2);
      if (lo_all & ~cr.w) {  // workgroup-uniform; rare (a new axis since the binning)
        Touch tr = tc;
        tr.tflag = rare->tflag;
        tr.touched = rare->touched;
        tr.nchunk = rare->nchunk;
        tr.rcov = rare->rcov;
        add_lower_tiles(tr, tl, tx, ty, tz, (lo_all | cr.w) & 7);
        if (k == 0) rare->chunk[w].w = lo_all | cr.w;
      }
      // stencil box of the chunk (empty chunk window: a 1-node box)
      int box = kFullBox;
      if (Mx && My && Mz)
        box = (__builtin_ctz(Mx)) | (__builtin_ctz(My) << 4) | (__builtin_ctz(Mz) << 8) | ((31 - __builtin_clz(Mx)) << 12) |
              ((31 - __builtin_clz(My)) << 16) | ((31 - __builtin_clz(Mz)) << 20);
      else
        box = 0;
      if (k == 0) {
        tc.cbox[w] = box;
        rare->tbox[t] = (cr.w & 8) ? kFullBox : box;  // tiles with several chunks: whole windows
      }
      if (tpos_e >= 0) rare->rbox[(size_t)tpos_e * kRecStride + k] = (cr.w & 8) ? kFullBox : box;
      if (cr.w & 8) box = kFullBox;
      if constexpr (kZeroBox) {  // only the nodes the scatter can reach and the store reads
        int lo[3], hi[3];
        box_unpack(box, lo, hi);
        const int n1 = hi[1] - lo[1] + 1, n2 = hi[2] - lo[2] + 1, n12 = n1 * n2;
        const int nvol = (hi[0] - lo[0] + 1) * n12;
        const float r12 = 1.0f / (float)n12, r2 = 1.0f / (float)n2;
        for (int qn = k; qn < nvol; qn += 256) {
          const int a = (int)(((float)qn + 0.5f) * r12), rem = qn - a * n12;
          const int bq = (int)(((float)rem + 0.5f) * r2), c = rem - bq * n2;
          const int node = ((lo[0] + a) * kFW1 + lo[1] + bq) * kFW2 + lo[2] + c;
#pragma unroll
          for (int ch = 0; ch < 4; ++ch) s_acc[ch * kFWin + node] = 0ull;
        }
        __syncthreads();  // zeroing before the adds
      }
      int ebits;
      frexpf(bmax, &ebits);
      const int S = bmax > 0.f ? 50 - ebits : 0;  // see k_p2g
      if (k < cnt) {
        if (win) {
          int bb[3];
          float fx[3], ww[3][3], dw[3][3];
          bspline(x, g.inv_dx, bb, fx, ww, dw);
          p2g_scatter<MAT, kFW1, kFW2, kFWin>(s_acc + ((b[0] - o0) * kFW1 + (b[1] - o1)) * kFW2 + (b[2] - o2), fx, ww,
                                              dw, v, C, m, nvt, g, dt, ldexp(1.0, S));
        } else {
          p2g_global<MAT>(x, v, C, m, nvt, g, dt, rare->gacc);
          *rare->esc = 1;
        }
      }
      {  // escape statistics (gsmpm_mpm_escapes): one atomic a wave with escapes; their tiles
        const unsigned long long eb = __ballot(k < cnt && !win);
        if (eb) {  // wave-uniform; rare.  (The tiles are marked here, after the scatter, not in its branch:
                   // there the code cost k_fused<metal> 1 % with no escape, profiles/r06/ab_esc_r06o.txt)
          if ((k & 63) == 0) atomicAdd(rare->esc_count, (unsigned)__popcll(eb));
          if (!kEscSweepAll && k < cnt && !win)
            mark_escape_tiles(rare->tflag, rare->touched, rare->nchunk + 1, rare->rcov, tl, ng, b[0], b[1], b[2]);
        }
      }
      __syncthreads();
      if (w == (int)blockIdx.x) stamp(SK, 4);
      if (tc.perm && k < cnt) tc.perm[(size_t)w * 256 + balanced_lane(s_rcnt, cnt, res, rrank)] = (unsigned char)q;
      if constexpr (kAtomicGrid) {  // the box into the dense accumulator, one lane per (node, channel)
        int lo[3], hi[3];
        box_unpack(box, lo, hi);
        const int n1 = hi[1] - lo[1] + 1, n2 = hi[2] - lo[2] + 1, n12 = n1 * n2;
        const int nvol = (hi[0] - lo[0] + 1) * n12;
        const float r12 = 1.0f / (float)n12, r2 = 1.0f / (float)n2;
        for (int e = k; e < 4 * nvol; e += 256) {
          const int qn = e >> 2, ch = e & 3;
          const int a = (int)(((float)qn + 0.5f) * r12), rem = qn - a * n12;
          const int bq = (int)(((float)rem + 0.5f) * r2), c = rem - bq * n2;
          const int wa = lo[0] + a, wb = lo[1] + bq, wc = lo[2] + c;
          const int node = (wa * kFW1 + wb) * kFW2 + wc;
          const int ix = o0 + wa, iy = o1 + wb, iz = o2 + wc;
          const float val = from_fixed32(s_acc[ch * kFWin + node], S);
          if (val != 0.f && (unsigned)ix < (unsigned)ng && (unsigned)iy < (unsigned)ng && (unsigned)iz < (unsigned)ng)
            unsafeAtomicAdd(reinterpret_cast<float*>(rare->gacc + (((size_t)ix * ng + iy) * ng + iz)) + ch, val);
        }
      } else {
        int lo[3], hi[3];
        box_unpack(box, lo, hi);
        const int n1 = hi[1] - lo[1] + 1, n2 = hi[2] - lo[2] + 1, n12 = n1 * n2;
        const int nvol = (hi[0] - lo[0] + 1) * n12;
        const float r12 = 1.0f / (float)n12, r2 = 1.0f / (float)n2;
        // the window's slot: the chunk's tile-order id (an ordered record carries it, k_chunk_order)
        const int cid = (cr.w & 16) ? (int)((unsigned)cr.w >> 5) : w;
        float4* dst = slots + (size_t)cid * kFWin;
        for (int qn = k; qn < nvol; qn += 256) {
          const int a = (int)(((float)qn + 0.5f) * r12), rem = qn - a * n12;
          const int bq = (int)(((float)rem + 0.5f) * r2), c = rem - bq * n2;
          const int node = ((lo[0] + a) * kFW1 + lo[1] + bq) * kFW2 + lo[2] + c;
          const int sl = kOwnerSlots ? slot_loc(lo[0] + a, lo[1] + bq, lo[2] + c) : node;
          float4 r;
          r.x = from_fixed32(s_acc[0 * kFWin + node], S);
          r.y = from_fixed32(s_acc[1 * kFWin + node], S);
          r.z = from_fixed32(s_acc[2 * kFWin + node], S);
          r.w = from_fixed32(s_acc[3 * kFWin + node], S);
          // write-through: a slot is read by other XCDs' grid updates, and a dirty
          // line left in this XCD's L2 would be written back by the end-of-kernel
          // release (k_fused 21.9 -> 18.2 us on the lego frame)
          wt_store4(dst + sl, r);
        }
      }
      __syncthreads();  // LDS reuse by the next chunk
    }
  }
  // end-of-launch housekeeping (no load of this launch depends on it)
  if (bin == 2) {  // the next launch re-bins into rare->bo: its counts and flags start at zero
    const BinOutF bo = rare->bo;
    for (int t = blockIdx.x * 256 + threadIdx.x; t <= tl.ntiles; t += gridDim.x * 256) {
      bo.count[t] = 0;
      if (t < tl.ntiles) bo.tflag[t] = 0;
    }
  }
  if (rare->esc_clr) {  // FOLD rotation (null outside it): escapes of launch r - 2, flag r - 3
    if (__builtin_amdgcn_readfirstlane(*rare->esc_old) != 0) {
      const size_t nn = (size_t)ng * ng * ng;
      for (size_t q = (size_t)blockIdx.x * 256 + threadIdx.x; q < nn; q += (size_t)gridDim.x * 256)
        rare->gacc_old[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *rare->esc_clr = 0;
  }
  stamp(SK, 1);
}

// The end of a FOLD step call: the escape accumulators that the call's last
// launches left dirty are zeroed and every rotation flag cleared, so the next
// call starts from clean buffers.  One workgroup (no flag is cleared while
// another workgroup could still test it); nothing to do in a call without
// escapes.
__global__ __launch_bounds__(1024) void k_fold_tail(int* __restrict__ flags, float4* __restrict__ g0,
                                                    float4* __restrict__ g1, float4* __restrict__ g2, int ng) {
  __shared__ int s_f[12];
  if (threadIdx.x < 12) s_f[threadIdx.x] = flags[threadIdx.x];
  __syncthreads();
  const size_t nn = (size_t)ng * ng * ng;
  bool dirty[3] = {false, false, false};
  for (int r = 0; r < 12; ++r) dirty[r % 3] = dirty[r % 3] || s_f[r] != 0;
  float4* gb[3] = {g0, g1, g2};
  for (int b = 0; b < 3; ++b)
    if (dirty[b])
      for (size_t q = threadIdx.x; q < nn; q += 1024) gb[b][q] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (threadIdx.x < 12 && s_f[threadIdx.x]) flags[threadIdx.x] = 0;
}

// Chunk ranges and stencil boxes of the 27 tiles whose windows reach tile
// (ti, tj, tk) -> LDS (lanes 0..26; caller syncs), in a cover record's layout:
// s_cov[2 e] = first chunk, s_cov[2 e + 1] = chunk count, s_bx[e] = box.
__device__ __forceinline__ void load_cover27(const ChunkIn& ck, const int* __restrict__ tbox, const FTiles& tl, int ti,
                                             int tj, int tk, int* s_cov, int* s_bx) {
  const int e = threadIdx.x;
  if (e < 27) {
    const int x = ti + e / 9 - 1, y = tj + (e / 3) % 3 - 1, z = tk + e % 3 - 1;
    int c0 = 0, nc = 0, bx = 0;
    if ((unsigned)x < (unsigned)tl.td0 && (unsigned)y < (unsigned)tl.td1 && (unsigned)z < (unsigned)tl.td2) {
      const int t = (x * tl.td1 + y) * tl.td2 + z;
      const int cnt = ck.count[t];
      c0 = ck.cbase[t];
      bx = tbox[t];
      nc = (cnt + kChunk - 1) / kChunk;
    }
    s_cov[2 * e] = c0;
    s_cov[2 * e + 1] = nc;
    s_bx[e] = bx;
  }
}

// The <= 8 window reads of owned node (l0, l1, l2) of a tile.  Per axis a node
// lies in its own tile's window and, when l < 3, in the lower neighbour's
// (l + T + 1 < T + 4), when l = T - 1 in the upper one's.  A read outside the
// covering tile's stencil box (nothing was scattered there this substep) is
// redirected to the all-zero slot, so the 8 loads stay unconditional.
struct NodeReads {
  int off[8];  // slot offsets (float4 units) of the first chunk of each covering tile
  int extra;   // bit e: covering tile e has further chunks
  int live;    // bit e: the node lies inside covering tile e's stencil box (some stencil may reach it)
};
// covering tile e of node (l0, l1, l2): its index in the 27-neighbourhood and the node's window offset there
__device__ __forceinline__ void node_cover(int l0, int l1, int l2, int e, int& ci, int& loc) {
  const int sec0 = l0 < 3 ? -1 : (l0 == kFT0 - 1 ? 1 : 0);
  const int sec1 = l1 < 3 ? -1 : (l1 == kFT1 - 1 ? 1 : 0);
  const int sec2 = l2 < 3 ? -1 : (l2 == kFT2 - 1 ? 1 : 0);
  const int a = (e >> 2) ? sec0 : 0, b = ((e >> 1) & 1) ? sec1 : 0, c = (e & 1) ? sec2 : 0;
  ci = (a + 1) * 9 + (b + 1) * 3 + (c + 1);
  loc = slot_loc(l0 - a * kFT0 + 1, l1 - b * kFT1 + 1, l2 - c * kFT2 + 1);
}
__device__ __forceinline__ void node_reads(int max_chunks, const int* s_cov, const int* s_bx, int l0,
                                           int l1, int l2, NodeReads& r) {
  const int sec0 = l0 < 3 ? -1 : (l0 == kFT0 - 1 ? 1 : 0);
  const int sec1 = l1 < 3 ? -1 : (l1 == kFT1 - 1 ? 1 : 0);
  const int sec2 = l2 < 3 ? -1 : (l2 == kFT2 - 1 ? 1 : 0);
  r.extra = 0;
  r.live = 0;
  // every LDS read first, unconditionally (ci is a valid neighbour index for
  // all e), then the tests as plain bit operations: with the reads behind
  // short-circuit tests the compiler branched around each one and waited on
  // each, 8 dependent LDS round trips in front of the slot loads
  int nc[8], bx[8], c0[8], ci[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int a = (e >> 2) ? sec0 : 0, b = ((e >> 1) & 1) ? sec1 : 0, c = (e & 1) ? sec2 : 0;
    ci[e] = (a + 1) * 9 + (b + 1) * 3 + (c + 1);
    nc[e] = s_cov[2 * ci[e] + 1];
    bx[e] = s_bx[ci[e]];
    c0[e] = s_cov[2 * ci[e]];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ax = e >> 2, ay = (e >> 1) & 1, az = e & 1;
    const int a = ax ? sec0 : 0, b = ay ? sec1 : 0, c = az ? sec2 : 0;
    const int w0 = l0 - a * kFT0 + 1, w1 = l1 - b * kFT1 + 1, w2 = l2 - c * kFT2 + 1;
    const int q = bx[e];
    const bool on = ((!ax) | (sec0 != 0)) & ((!ay) | (sec1 != 0)) & ((!az) | (sec2 != 0)) & (nc[e] > 0) &
                    (w0 >= (q & 15)) & (w1 >= ((q >> 4) & 15)) & (w2 >= ((q >> 8) & 15)) &
                    (w0 <= ((q >> 12) & 15)) & (w1 <= ((q >> 16) & 15)) & (w2 <= ((q >> 20) & 15));
    const int loc = slot_loc(w0, w1, w2);
    r.off[e] = on ? c0[e] * kFWin + loc : max_chunks * kFWin;
    r.extra |= (on & (nc[e] > 1)) ? (1 << e) : 0;
    r.live |= on ? (1 << e) : 0;
  }
}
__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}
// the further chunks of covering tiles with several (tiles of > 256
// particles: a few in the 100k lego frame, most of the 240k one's).  The
// second chunks of the 8 covering tiles are read in batches of 4 (a batch's
// loads in flight together, the zero slot for a tile without one), then the third and
// later ones (tiles of > 512 particles) one by one.  Until round 5 every extra
// chunk was a load and its wait inside the loop: one round trip each.
// one dword a lane, global -> LDS (LDS-DMA): lane l's word lands at
// lds_base + 4 l (lds_base wave-uniform), tracked by vmcnt like a load
__device__ __forceinline__ void glds4(const int* src, int* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 4, 0, 0);
}
// a window slot by its float4 offset, addressed as the slots' SGPR base plus a
// 32-bit byte offset (global_load saddr form: one VGPR per address, not a
// 64-bit pair; the slot array is < 4 GiB, checked where it is sized)
__device__ __forceinline__ float4 ld_slot(const float4* __restrict__ slots, int off) {
  return *(const float4*)((const char*)slots + (unsigned)off * 16u);
}
#ifndef GSMPM_EXTRA_BATCH
#define GSMPM_EXTRA_BATCH 4
#endif
constexpr int kExtraBatch = GSMPM_EXTRA_BATCH;  // second-chunk loads in flight (8: VGPR spills)
__device__ __forceinline__ void node_extra(const float4* __restrict__ slots, const int* s_cov, int l0,
                                           int l1, int l2, int extra2, int zero, float4& acc) {
  // (the offsets recomputed from the LDS cover table: keeping node_reads'
  // 8 offsets live across the first batch spilled VGPRs)
  int o2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    int ci, loc;
    node_cover(l0, l1, l2, e, ci, loc);
    o2[e] = ((extra2 >> e) & 1) ? (s_cov[2 * ci] + 1) * kFWin + loc : zero;
  }
#pragma unroll
  for (int h = 0; h < 8; h += kExtraBatch) {
    float4 u[kExtraBatch];
#pragma unroll
    for (int e = 0; e < kExtraBatch; ++e) u[e] = ld_slot(slots, o2[h + e]);
#pragma unroll
    for (int e = 0; e < kExtraBatch; ++e) add4(acc, u[e]);
    __builtin_amdgcn_sched_barrier(0);  // (else the batches merge: 8 in flight, and spills)
  }
  int extra = extra2;  // (a tile of <= 512 particles: no iteration)
  while (extra) {
    const int e = __builtin_ctz(extra);
    extra &= extra - 1;
    int ci, loc;
    node_cover(l0, l1, l2, e, ci, loc);
    for (int w = s_cov[2 * ci] + 2; w < s_cov[2 * ci] + s_cov[2 * ci + 1]; ++w) add4(acc, ld_slot(slots, w * kFWin + loc));
  }
}

// Grid update of the fused pipeline: kGridParts one-wave workgroups per
// touched tile (64 consecutive owned nodes each), one owned node per lane (all
// 8 window reads in flight); a scene's ~900 touched tiles run in one round.
// Measured (lego frame): one 448-lane workgroup per tile 17.4 us, two 224-lane
// 12.45, four 112-lane 12.1, seven 64-lane 12.2 with k_fused unaffected
// (sim 3.27-3.28 against 3.29-3.32 ms/frame for two).
// esc_in: some particle scattered through gacc in the P2G this update consumes
// -> every tile, plus gacc (re-zeroed).  esc_clear: the flag the next P2G
// raises.  zc / zf (optional): the counts / touched flags the next binning
// launch accumulates into.
#ifndef GSMPM_GRID_PARTS
#define GSMPM_GRID_PARTS 7
#endif
constexpr int kGridParts = GSMPM_GRID_PARTS;  // workgroups per touched tile
constexpr int kGridT = kFTN / kGridParts;     // lanes per grid workgroup
// Nodes that no particle stencil can reach keep whatever v_out they held: a
// node outside every covering chunk's stencil box (the union of its
// particles' stencils at this P2G, which the next G2P gathers from unmoved)
// is read by no G2P before the next grid update rewrites it.  Every node
// inside a box is stored, massless or not, so a stencil node of a particle
// too light to register in the fixed-point sums (below 2^-51 of its chunk's
// heaviest: its mass rounds to zero) reads 0 as from the reference's reset
// grid (utils.py:177-183), not a stale value (round 4 skipped every massless
// node; test_gpu_mpm.py::test_heterogeneous_masses).  GSMPM_GRID_SKIP0=0
// stores every node of the touched tiles, =2 only nodes with mass (round 4's
// form, A/B).
#ifndef GSMPM_GRID_SKIP0
#define GSMPM_GRID_SKIP0 1
#endif
constexpr bool kGridSkip0 = GSMPM_GRID_SKIP0 != 0;
// GSMPM_GVEL_STORE (A/B): the v_out store of k_grid_f plain (0), streaming nt
// (1) or write-through sc1 (2; round 2: the gap after k_grid_f 2.6 -> 1.5 us,
// k_grid_f +0.8 us)
#ifndef GSMPM_GVEL_STORE
#define GSMPM_GVEL_STORE 0
#endif
constexpr int kGvelStore = GSMPM_GVEL_STORE;
// SLAB: a slab rank's grid pass (SlabWin hooks); the single-domain form is
// compiled without them -- their ~20 argument dwords pushed the kernel past
// the SGPR budget: 21 spilled SGPRs (21 v_writelane at the start, 26
// v_readlane restores, ~13 % of the ~350 VALU instructions a wave issues)
// against 4 now; k_grid_f 12.06 -> 11.67 us in the lego frame (5
// interleaved rounds, profiles/r05/ab/ab_rare_args_pk_r05k.txt)
// XCD-grouped work order (round 6).  Workgroup b runs on XCD b % 8, and each
// XCD has its own L2.  A window slot is read by the grid update of its own
// tile and of the upper neighbours whose low nodes it covers, and a tile's
// seven parts read one cover record; in the plain order (work item b: tile
// b / 7, part b % 7) the seven parts of a tile land on seven XCDs and
// neighbouring tiles on others, so each line is fetched once per XCD that
// reads it.  Here a tile's parts run on one XCD, and kGridGroup consecutive
// touched tiles (the touched list is in tile order: z-neighbours, whose
// windows share lines, are adjacent) go to one XCD before the next XCD's
// group.  tools/grid_f_bytes.py models the lego launch at 20.5 MB fetched in
// the plain order (FETCH_SIZE: 21.3 MB) and 10.9 MB grouped by 16.  The grid
// is a multiple of 8 workgroups (launch_grid_f).  GSMPM_GRID_GROUP=0: the
// plain order (A/B).
#ifndef GSMPM_GRID_GROUP
#define GSMPM_GRID_GROUP 16
#endif
constexpr int kGridGroup = GSMPM_GRID_GROUP;
// work item it of workgroup b (grid stride S): touched position P, part
// (P never decreases with it, so a workgroup stops at the first P past the count)
__device__ __forceinline__ void grid_work(int b, int it, int S, int& P, int& part) {
  if constexpr (kGridGroup == 0) {
    const int wt = b + it * S;
    P = wt / kGridParts;
    part = wt - P * kGridParts;
  } else {
    const int x = b & 7, m = (b >> 3) + it * (S >> 3);
    const int u = m / kGridParts, k = u / kGridGroup;
    part = m - u * kGridParts;
    P = (k * 8 + x) * kGridGroup + (u - k * kGridGroup);
  }
}
template <bool SLAB>
__global__ __launch_bounds__(kGridT) __attribute__((amdgpu_waves_per_eu(7, 8))) void k_grid_f(GridDims g, FTiles tl, ChunkIn ck, const int* __restrict__ tbox,
                                                    const float4* __restrict__ slots, float4* __restrict__ gacc,
                                                    float4* __restrict__ gvel, const BcTable* __restrict__ bct,
                                                    GridStep gs, const int* __restrict__ esc_in,
                                                    int* __restrict__ esc_clear, int* __restrict__ zc,
                                                    int* __restrict__ zf, SlabWin sw) {
  sim_prio();
  stamp(3, 0);
  // a slab's grid update runs as two passes (window tiles first, so their
  // partials can travel while the rest updates): the flag and the zeroing go
  // with the second
  const int pass = SLAB ? sw.pass : 0;
  // Every first load of the workgroup is issued here, together, before any
  // store: the escape flag, the touched count, the first touched tile (its
  // index clamped) and that tile's cover record -- its 27 neighbours' chunk
  // ranges (from the binning) and stencil boxes (published by this
  // substep's k_fused), so the slot addresses need no hop through the tile
  // tables.  Round 5 first had the flag and count after the zeroing stores
  // below, which the compiler may not hoist loads over (the pointers could
  // alias): three dependent scalar round trips before the first record load.
  int P0, part0;
  grid_work(blockIdx.x, 0, gridDim.x, P0, part0);
  const int i0 = min(P0, tl.ntiles - 1);
  // (the empty asm takes the three pointers into SGPRs at once, so their
  // kernel-argument loads come in the first batch and the three scalar loads
  // below leave together: one round trip, not two behind each other)
  const int* esc_p = esc_in;
  const int* cnt_p = ck.nchunk;
  const int* tch_p = ck.touched;
  asm volatile("" : "+s"(esc_p), "+s"(cnt_p), "+s"(tch_p));
  const bool recs = ck.rcov != nullptr && !kAtomicGrid;
  const int le = threadIdx.x;  // lane: record entry
  // Cover records reach LDS by LDS-DMA (global_load_lds: no VGPR holds
  // them): buffer b of s_rec / s_box holds the tile being updated, and at the
  // top of each iteration the NEXT tile's record and id are requested into
  // the other buffer, so a workgroup owning several tiles (config D: ~27 a
  // launch) pays one round trip a tile (its slot loads) instead of two.  A
  // record is 64 dwords (27 {first chunk, count} pairs + the "none" flag at
  // dword 54) and its boxes 32; lane le moves dword le of each (the boxes'
  // upper half a harmless copy of the lower).
  __shared__ int s_rec[2][64];
  __shared__ int s_box[2][64];
  __shared__ int s_tn[2];
  // (wave 0's lanes only: the DMA writes lds_base + 4 x lane-in-wave)
  if (recs && threadIdx.x < 64) {
    glds4(reinterpret_cast<const int*>(ck.rcov) + (size_t)i0 * 2 * kRecStride + le, &s_rec[0][0]);
    glds4(ck.rbox + (size_t)i0 * kRecStride + (le & 31), &s_box[0][0]);
  }
  typedef const int __attribute__((address_space(1)))* gint_p;  // global, not flat (flat loads count in lgkmcnt too)
  // (uniform words: readfirstlane keeps them in SGPRs, not three VGPRs live across the tile loop)
  const int esc0 = __builtin_amdgcn_readfirstlane(*(gint_p)esc_p);
  const int cnt0 = __builtin_amdgcn_readfirstlane(((gint_p)cnt_p)[1]);
  const int T0 = __builtin_amdgcn_readfirstlane(((gint_p)tch_p)[i0]);
  const int ng = g.ng;
  const bool esc = esc0 != 0;            // the escape accumulator holds sums: add it to the owned nodes
  const bool all = esc && kEscSweepAll;  // (A/B) every tile, not the touched ones
  const int ntouch = all ? tl.ntiles : cnt0;  // tiles to update
  const bool pre = recs && !all;  // workgroup-uniform: records in LDS, the next one prefetched
  int b = 0;
  for (int it = 0;; ++it, b ^= 1) {
    int P, part;
    grid_work(blockIdx.x, it, gridDim.x, P, part);
    if (P >= ntouch) break;  // workgroup-uniform
    if constexpr (!kAtomicGrid) {
      // this tile's DMA (issued a tile ago, or in the prologue) has landed;
      // readers of the other buffer are done.  The wait is explicit: the
      // compiler's own waits for LDS-DMA did not cover every read of these
      // arrays (the slab test caught stale records), and a one-wave
      // workgroup's barrier compiles to nothing.  What else it waits for is
      // the previous tile's v_out stores (L2 write acks, not an HBM trip).
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int pn, partn;
      grid_work(blockIdx.x, it + 1, gridDim.x, pn, partn);
      if (pre && pn < ntouch && threadIdx.x < 64) {  // workgroup-uniform (kGridT = 64: one wave)
        glds4(reinterpret_cast<const int*>(ck.rcov) + (size_t)pn * 2 * kRecStride + le, &s_rec[b ^ 1][0]);
        glds4(ck.rbox + (size_t)pn * kRecStride + (le & 31), &s_box[b ^ 1][0]);
        if (le == 0) glds4(ck.touched + pn, &s_tn[b ^ 1]);
      }
    }
    int* s_cov = s_rec[b];
    int* s_bx = s_box[b];
    const int q = threadIdx.x + part * kGridT;
    const int l0 = q / (kFT1 * kFT2), l1 = (q / kFT2) % kFT1, l2 = q % kFT2;
    const int T = all ? P : it == 0 ? T0 : pre ? s_tn[b] : ck.touched[P];
    if ((unsigned)T >= (unsigned)tl.ntiles) continue;  // workgroup-uniform; never taken (P < count)
    int ti, tj, tk;
    ftile_decode(tl, T, ti, tj, tk);
    if (SLAB && pass != 0 && slab_tile_in_window(sw, ti) != (pass == 1)) continue;  // workgroup-uniform
    if constexpr (!kAtomicGrid) {
      if (it == 0) stamp(3, 2);
      // a tile k_fused appended (add_lower_tiles) has no record: "none" flag
      const bool tables = !pre || s_cov[54] != 0;  // workgroup-uniform
      if (tables) {
        load_cover27(ck, tbox, tl, ti, tj, tk, s_cov, s_bx);
        __syncthreads();
      }
    }
    if (it == 0) stamp(3, 3);
    const int i = ti * kFT0 + l0, j = tj * kFT1 + l1, k = tk * kFT2 + l2;
    if ((unsigned)i < (unsigned)ng && (unsigned)j < (unsigned)ng && (unsigned)k < (unsigned)ng) {
      const size_t idx = ((size_t)i * ng + j) * ng + k;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      bool reach = true;  // some stencil box covers the node (the atomic A/B form: mass only)
      if constexpr (kAtomicGrid) {  // the node's whole sum, added by the chunks' atomics
        a = gacc[idx];
        if (a.x != 0.f || a.y != 0.f || a.z != 0.f || a.w != 0.f) gacc[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        NodeReads r;
        node_reads(tl.max_chunks, s_cov, s_bx, l0, l1, l2, r);
        reach = r.live != 0;
        float4 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ld_slot(slots, r.off[e]);
#pragma unroll
        for (int e = 0; e < 8; ++e) add4(a, v[e]);
        if (r.extra) node_extra(slots, s_cov, l0, l1, l2, r.extra, tl.max_chunks * kFWin, a);
        if (esc) {  // the nodes an escape wrote lie in touched tiles (mark_escape_tiles); zero what was written
          const float4 e = gacc[idx];
          add4(a, e);
          if (all || e.x != 0.f || e.y != 0.f || e.z != 0.f || e.w != 0.f) gacc[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      bool inrect = false;
      if constexpr (SLAB) {
        const int sww = sw.W ? slab_window_of(sw, i) : -1;
        inrect = sww >= 0 && (unsigned)(j - sw.y0[sww]) < (unsigned)sw.ny[sww] &&
                 (unsigned)(k - sw.z0[sww]) < (unsigned)sw.nz[sww];
        if (sww >= 0 && !inrect && a.w != 0.f) *sw.oob = 1;
        if (inrect)  // a window node: this rank's partial, totalled after the exchange (k_win_update)
          sw.part[sww][((size_t)(i - sw.a[sww]) * sw.ny[sww] + (j - sw.y0[sww])) * sw.nz[sww] + (k - sw.z0[sww])] = a;
      }
      if (inrect) {
      } else if (!kGridSkip0 || a.w != 0.f || (reach && !kAtomicGrid && GSMPM_GRID_SKIP0 == 1)) {
        if constexpr (kGvelStore == 1)
          nt_store4(gvel + idx, node_update(a, i, j, k, g, gs, bct));
        else if constexpr (kGvelStore == 2)
          wt_store4(gvel + idx, node_update(a, i, j, k, g, gs, bct));
        else
          gvel[idx] = node_update(a, i, j, k, g, gs, bct);
      }
    }
    if (it == 0) stamp(3, 4);
  }
  // the zeroing for the next launches, after the tiles: its stores are not
  // in front of any wait above
  if (blockIdx.x == 0 && threadIdx.x == 0 && pass != 1) *esc_clear = 0;
  if (zc && pass != 1) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t <= tl.ntiles; t += gridDim.x * blockDim.x) {
      zc[t] = 0;
      if (t < tl.ntiles) zf[t] = 0;
    }
  }
  stamp(3, 1);
}

// bin every particle by its current x (set_particles / resort / set x)
__global__ __launch_bounds__(256) void k_bin_all_f(Particles ps, GridDims g, BinOutF bo) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < ps.count()) {
    float x[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = ps.ld(PX + d, p);
    int tc[3];
    const int t = ftile_of(x, g, bo.tl, tc);
    bo.ptile[p] = t;
    bo.pslot[p] = reserve_f(bo, t, 1);
  }
}
