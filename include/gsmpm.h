/*
 * gsmpm.h -- C-ABI of the MI355X-native PhysGaussian hot path (libgsmpm.so).
 *
 * Plain C types only: device pointers are `float*`/`int32_t*` allocated by
 * the caller (e.g. torch tensors' data_ptr()), streams are `void*`
 * (hipStream_t).  Every entry point returns 0 on success or a negative
 * status; gsmpm_last_error() then holds a thread-local message.
 *
 * Each declaration names the reference interface it replaces
 * (ranrandy/gaussian-splatting-mpm @ 2024-12-18, file:line).
 */
#ifndef GSMPM_H
#define GSMPM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSMPM_OK 0
#define GSMPM_EINVAL -1
#define GSMPM_EHIP -2
#define GSMPM_ESTATE -3
#define GSMPM_ESPACE -4  /* a caller-owned workspace is too small (gsmpm_raster_forward_ws) */

/* ------------------------------------------------------------ common --- */
const char* gsmpm_last_error(void);
int gsmpm_version(void);

/* --------------------------------------------------------------- MPM ---
 * Replaces mpm_solver.MPM_Simulator (mpm_solver/solver.py:9-177) with its
 * MPM_model / MPM_state (mpm_solver/model.py:6-132).
 */
typedef struct gsmpm_mpm gsmpm_mpm;

#define GSMPM_MAT_JELLY 0
#define GSMPM_MAT_METAL 1
#define GSMPM_MAT_SAND 2
#define GSMPM_MAT_FOAM 3

/* flags */
#define GSMPM_FLAG_JELLY_FCR 1u   /* fix SURVEY F3: run FCR elasticity for jelly (utils.py:37-38) */
#define GSMPM_FLAG_KEEP_GRID 2u   /* keep m / m*v of the last substep readable (debug, slower) */
#define GSMPM_FLAG_NO_GRAPH 4u    /* launch substeps eagerly instead of through a cached hipGraph */
#define GSMPM_FLAG_NO_SORT 8u     /* keep particles in input order (no spatial sort) */
#define GSMPM_FLAG_PHASED 16u     /* per-phase substep (P2G, grid, G2P, binning: 4 launches) instead of the
                                     fused G2P2G pipeline (2 launches); also implied by KEEP_GRID */

/* substep pipelines (gsmpm_mpm_pipeline) */
#define GSMPM_PIPE_PHASED 0
#define GSMPM_PIPE_FUSED 1

typedef struct {
  int32_t n_particles;
  int32_t n_grid;               /* MPMParams.n_grid (arguments/__init__.py:66) */
  double grid_extent;           /* MPMParams.grid_extent */
  int32_t material;             /* GSMPM_MAT_*; model.py:24-31 */
  double E, nu, density;        /* model.py:42-44, 100-102 */
  double gravity[3];            /* model.py:32 */
  double yield_stress;          /* 0.005, model.py:55-56 */
  double hardening, xi;         /* 1, 1, model.py:57-58 */
  double plastic_viscosity;     /* 0.008, model.py:59 */
  double friction_angle_deg;    /* 25, model.py:48 */
  uint32_t flags;
} gsmpm_mpm_params;

/* MPM_Simulator.__init__ -> MPM_model.__init__ (model.py:8-22) */
int gsmpm_mpm_create(const gsmpm_mpm_params* params, gsmpm_mpm** out);
int gsmpm_mpm_destroy(gsmpm_mpm* h);

/* MPM_state.__init__ (model.py:78-122): x [N,3] grid space, cov6 [N,6]
 * (becomes particle_init_cov and particle_cov), vol [N]; v [N,3] or NULL
 * (MPM_state_opt init_vel, model.py:160-167).  Device pointers, f32. */
int gsmpm_mpm_set_particles(gsmpm_mpm* h, const float* x, const float* cov6, const float* vol,
                            const float* v_or_null, void* stream);

/* Boundary conditions (mpm_solver/boundary_conditions.py, solver.py:110-167).
 * Each returns (>=0) a bc id; ids index the bit of the per-substep activity mask.
 *   fixed_cube  -> BasicBC.apply           (boundary_conditions.py:23-27)
 *   impulse     -> ImpulseBC.apply         (boundary_conditions.py:41-45)
 *   plane       -> MPM_Collider.collide    (collider.py:13-44), always active;
 *                  normal is normalised in f64 as solver.py:153-154 does. */
int gsmpm_mpm_add_fixed_cube(gsmpm_mpm* h, const double center[3], const double size[3]);
int gsmpm_mpm_add_impulse(gsmpm_mpm* h, const double center[3], const double size[3], const double force[3],
                          double substep_dt);
int gsmpm_mpm_add_plane_collider(gsmpm_mpm* h, const double point[3], const double normal[3], double friction);

/* MPM_Simulator.p2g2p (solver.py:27-52) x n_substeps.  bc_active[s] holds
 * the activity bits of substep s, decided by the caller from the f64 host
 * clock exactly as BasicBC.isActive (boundary_conditions.py:30-31); NULL =
 * all active.  Asynchronous on `stream`.  Returns GSMPM_ESTATE (and launches
 * nothing) once an earlier call's substeps produced non-finite (NaN / Inf)
 * particle state: a position, or a scatter input of P2G -- mass, velocity
 * (after an impulse), C or the stress term -- while x may still be finite
 * (SURVEY 5's per-frame check; the kernels set a sticky host-mapped word,
 * read here without a sync: the error surfaces at the call after the frame
 * that produced it, or at gsmpm_mpm_check_finite). */
int gsmpm_mpm_step(gsmpm_mpm* h, float dt, int32_t n_substeps, const uint32_t* bc_active, void* stream);
/* Synchronizes `stream`, then GSMPM_ESTATE if any substep so far produced a
 * non-finite particle state (position, mass, velocity, C or stress; clear
 * != 0 resets the word; set_particles does too), else GSMPM_OK.  No
 * reference counterpart. */
int gsmpm_mpm_check_finite(gsmpm_mpm* h, int32_t clear, void* stream);

/* ------------------------------------------------- multi-GPU slabs ---
 * SURVEY 8(e); no reference counterpart (the reference is one device,
 * main.py:28): the substep of mpm_solver/solver.py:27-52 sharded by spatial
 * slab along grid axis 0, one rank per GPU (csrc/slab.h, gsmpm/dist.py).
 *
 * A transport moves the boundary-node partial sums (every substep) and the
 * migrating particles (every `interval` substeps) between neighbouring ranks:
 *   GSMPM_XPORT_RCCL      comm is an ncclComm_t (gsmpm_rccl_comm_init):
 *                         grouped ncclSend/ncclRecv with ranks r-1 / r+1 on
 *                         a stream of the simulator's, overlapping the
 *                         interior grid update;
 *   GSMPM_XPORT_CALLBACK  fn(user, n, peers, send, send_bytes, recv,
 *                         recv_bytes) is called on the host after the stream
 *                         is synchronised, with pinned HOST copies of the
 *                         buffers (tests: gloo, several ranks on one GPU).
 * Both sides of every pair post the same sizes in the same order. */
#define GSMPM_XPORT_NONE 0
#define GSMPM_XPORT_RCCL 1
#define GSMPM_XPORT_CALLBACK 2
typedef int (*gsmpm_exchange_fn)(void* user, int32_t n, const int32_t* peers, void* const* send,
                                 const size_t* send_bytes, void* const* recv, const size_t* recv_bytes);
typedef struct {
  int32_t kind;          /* GSMPM_XPORT_* */
  int32_t rank, world;
  void* comm;            /* ncclComm_t (RCCL) */
  gsmpm_exchange_fn fn;  /* CALLBACK */
  void* user;
} gsmpm_transport;

/* RCCL communicator for the slab exchange (ncclGetUniqueId / ncclCommInitRank
 * of the RCCL already loaded in the process, dlopen'ed -- torch's when torch
 * is imported).  id is 128 bytes: rank 0 creates it, every rank receives it
 * (e.g. torch.distributed broadcast) and calls comm_init on its own GPU. */
int gsmpm_rccl_unique_id(uint8_t id[128]);
int gsmpm_rccl_comm_init(const uint8_t id[128], int32_t rank, int32_t world, void** comm);
int gsmpm_rccl_comm_destroy(void* comm);

/* Make `h` (created with n_particles = this rank's particle CAPACITY) rank
 * `rank` of a `world`-slab domain owning grid planes [lo, hi) of axis 0;
 * particles may drift `margin` planes between migrations, which happen every
 * `interval` substeps inside gsmpm_mpm_slab_step.  Call before
 * gsmpm_mpm_slab_set_particles.  Neighbouring slabs must be >= 2*margin+2
 * planes thick. */
int gsmpm_mpm_slab_init(gsmpm_mpm* h, int32_t rank, int32_t world, int32_t lo, int32_t hi, int32_t margin,
                        int32_t interval);
/* This rank's initial particles (n <= capacity) with their global ids
 * (device int32[n]); otherwise as gsmpm_mpm_set_particles. */
int gsmpm_mpm_slab_set_particles(gsmpm_mpm* h, int32_t n, const float* x, const float* cov6, const float* vol,
                                 const float* v_or_null, const int32_t* gid, void* stream);
/* n_substeps substeps of the slab (bc masks as gsmpm_mpm_step), window
 * exchange every substep and particle migration every `interval` substeps
 * through `xp`, all on the device (with RCCL one captured graph per call:
 * counts never visit the host inside the call).  Migration payloads have a
 * fixed capacity, grown between calls; leavers beyond it stay for a later
 * migration.  Returns GSMPM_ESTATE if a particle drifted past the margin or a
 * window node outside the exchanged rect got mass (contributions were not
 * exchanged: the state is invalid) or a slab would exceed its capacity: every
 * rank's record goes to every rank at the end of the call, so all ranks return
 * it from the same call, with the same message naming the rank at fault. */
int gsmpm_mpm_slab_step(gsmpm_mpm* h, float dt, int32_t n_substeps, const uint32_t* bc_active_mask,
                        const gsmpm_transport* xp, void* stream);
/* current particle count of this rank (changes with migration) */
int gsmpm_mpm_count(gsmpm_mpm* h);
/* global ids of this rank's particles, in the order gsmpm_mpm_get returns rows */
int gsmpm_mpm_get_gid(gsmpm_mpm* h, int32_t* out, void* stream);
/* {migrations, particles migrated (sent), lo, hi, margin, interval, window planes, capacity,
 *  leavers deferred (payload full), migration payload capacity, host syncs inside
 *  gsmpm_mpm_slab_step (one per call, plus one on the first call after set_particles),
 *  step calls} */
int gsmpm_mpm_slab_stats(gsmpm_mpm* h, int64_t out12[12]);
/* The yz rect of each window that the exchange moves, agreed by the two ranks of
 * the bound at every migration: {y0, ny, z0, nz} of the lower window, then of the
 * upper one (ny = nz = 0: nothing to exchange; before the first slab_step, the
 * whole cross-section). */
int gsmpm_mpm_slab_rects(gsmpm_mpm* h, int32_t out8[8]);
/* Re-cutting the slabs ("rebalance per frame"; on by default,
 * tolerance 0.05): at the end of a step call, when the most loaded slab holds
 * more than (1 + tolerance) x the mean particle count, every rank moves the
 * bounds to the count quantiles of all ranks' base-plane histograms (the same
 * records on every rank: the same bounds), each bound staying inside its old
 * neighbouring slabs; the next call opens with the migration to them. */
int gsmpm_mpm_slab_set_rebalance(gsmpm_mpm* h, int32_t on, float tolerance);
/* This rank's weight in the re-cut (default 1; > 0): the bounds move to the
 * quantiles that give rank r the share w_r / sum(w) of the particles, and a
 * rank holding more than (1 + tolerance) x its share triggers the re-cut.  A
 * rank with other work per frame takes a smaller share: the rank that renders
 * the gathered frame (bench.py, SlabDomain.set_render_share) sets
 * w = (W s - (W - 1) r) / (W s + r) from its simulation time s at an even
 * share and its render time r (W = world size), so its sim + render matches
 * the other ranks' sim when the sim time is linear in the particle count.
 * Carried in each rank's record (the next step call's), so every rank sees
 * every weight.  No reference counterpart. */
int gsmpm_mpm_slab_set_weight(gsmpm_mpm* h, float weight);
/* The current bounds of every slab, out[world + 1] (before the first step call
 * only this rank's own two, the rest -1), and the re-cuts made so far. */
int gsmpm_mpm_slab_bounds(gsmpm_mpm* h, int32_t* out, int32_t n, int64_t* rebalances);

/* Re-sort particle storage into Morton order of the current cells now (only
 * summation order changes; rows stay in caller order).  interval >= 0 also sets
 * how many substeps gsmpm_mpm_step lets pass between automatic re-sorts
 * (0 = never; default 100).  No counterpart in the reference. */
int gsmpm_mpm_resort(gsmpm_mpm* h, int32_t interval, void* stream);

/* Fused pipeline: substeps between re-binnings of the particles into tiles
 * (at most; default 20 for stress-free materials, 25 for stress-bearing ones; any
 * value is correct -- particles that moved more than one cell
 * since their binning take a slower global path).  Fixes the spacing: the
 * adaptive choice (gsmpm_mpm_rebin_state) is turned off.  No counterpart in
 * the reference (its p2g2p has no binning, solver.py:27-52). */
int gsmpm_mpm_set_rebin_interval(gsmpm_mpm* h, int32_t substeps);
/* Fused pipeline, one domain: with GSMPM_REBIN_AUTO=1 in the environment at
 * create (off by default: DESIGN.md §3.4), the re-binnings of each step call
 * adapt to the particles' speed (gsmpm_mpm_set_rebin_interval fixes the
 * spacing again): from the fastest
 * velocity component the previous call ended with (copied to pinned memory
 * without a sync) plus what gravity adds, enough re-binnings that no
 * particle moves more than 0.8 cell between two -- a particle that leaves
 * its chunk's window makes the next grid update sweep every tile -- and at
 * least one per rebin_interval substeps.  out3 = {rebin_interval, auto
 * (0/1), re-binnings chosen for the last call (0: from rebin_interval)};
 * *vmax (may be null) = the last fastest velocity component seen.  No
 * reference counterpart (the reference does not bin, solver.py:27-52). */
int gsmpm_mpm_rebin_state(gsmpm_mpm* h, int32_t* out3, float* vmax);
/* GSMPM_PIPE_FUSED or GSMPM_PIPE_PHASED: the pipeline gsmpm_mpm_step runs now. */
int gsmpm_mpm_pipeline(gsmpm_mpm* h);
/* 1 when the fused pipeline folds each substep's grid update into the next
 * k_fused launch (one launch per substep; a k_grid_f launch only after a
 * re-binning): GSMPM_FOLD=1 in the environment at create, off by default
 * (measured slower); 0 otherwise (the default, the per-phase
 * pipeline, slabs).  The grid update it folds is utils.py:177-183 +
 * solver.py:41-46; without escapes the results are bit-identical either way. */
int gsmpm_mpm_folded(gsmpm_mpm* h);
/* Fused pipeline diagnostics: the particle scatters since set_particles (or
 * the last clear) that left their chunk's window -- they took the global
 * float-atomic path, and the next grid update evaluates every node they may
 * reach -- (particles binned outside the grid count every substep).
 * Synchronizes `stream`.  0 on the per-phase pipeline.  No reference
 * counterpart (the reference scatters every particle with atomics,
 * utils.py:89-134). */
int gsmpm_mpm_escapes(gsmpm_mpm* h, int32_t clear, int64_t* out, void* stream);

/* MPM_Simulator.postprocess (solver.py:135-137): compute_cov_from_F and
 * compute_R_from_F (utils.py:376-433). */
int gsmpm_mpm_postprocess(gsmpm_mpm* h, void* stream);

/* Field readback / write in the reference layout (Taichi to_torch shapes):
 * rows follow the caller's original particle order. */
#define GSMPM_FIELD_X 0        /* particle_xyz      [N,3]   */
#define GSMPM_FIELD_V 1        /* particle_vel      [N,3]   */
#define GSMPM_FIELD_C 2        /* particle_C        [N,3,3] */
#define GSMPM_FIELD_F_TRIAL 3  /* particle_F_trial  [N,3,3] */
#define GSMPM_FIELD_COV 4      /* particle_cov      [6N]    */
#define GSMPM_FIELD_INIT_COV 5 /* particle_init_cov [6N]    */
#define GSMPM_FIELD_R 6        /* particle_R        [N,3,3] */
#define GSMPM_FIELD_MASS 7     /* particle_mass     [N]     */
#define GSMPM_FIELD_VOL 8      /* particle_vol      [N]     */
#define GSMPM_FIELD_MU 9       /* mpm_model.mu      [N]     */
#define GSMPM_FIELD_LAM 10     /* mpm_model.lam     [N]     */
#define GSMPM_FIELD_YIELD 11   /* mpm_model.yield_stress [N] */
#define GSMPM_FIELD_COUNT 12
int gsmpm_mpm_field_width(int32_t field);
int gsmpm_mpm_get(gsmpm_mpm* h, int32_t field, float* out, void* stream);
int gsmpm_mpm_set(gsmpm_mpm* h, int32_t field, const float* in, void* stream);

/* Grid readback [n^3] / [n^3,3] (grid_mass / grid_v_in / grid_v_out,
 * model.py:117-121).  mass and v_in need GSMPM_FLAG_KEEP_GRID. */
#define GSMPM_GRID_MASS 0
#define GSMPM_GRID_V_IN 1
#define GSMPM_GRID_V_OUT 2
int gsmpm_mpm_get_grid(gsmpm_mpm* h, int32_t which, float* out, void* stream);

/* Fused frame output (main.py:310-313 + render_frame 139-146), f32 as torch does it:
 * means_out[N,3] = (x - extent/2)/s + c            (grid2world, transform_utils.py:18-21)
 *                  and, if render_space != 0, then c + (means - 1)/1.0
 *                  (undoshift2center111 + undotransform2origin with scale 1.0);
 * cov_out[N,6]   = cov / (s*s).   Rows in original particle order. */
int gsmpm_mpm_world_outputs(gsmpm_mpm* h, float scale, const float center[3], int32_t render_space,
                            float* means_out, float* cov_out, void* stream);

/* Measurement: run n substeps eagerly on `stream`, each kernel launched with
 * hipExtLaunchKernel start/stop events (stamped by its own dispatch, the
 * interval rocprofv3 reports); kernel_ms[0..3] = summed time of k_p2g,
 * k_grid, k_g2p and the binning (k_finish_bins, or k_scan_tiles..k_scatter)
 * -- for the fused pipeline {k_fused, k_grid_f, binning, 0}.
 * Synchronises `stream`. */
int gsmpm_mpm_profile_substeps(gsmpm_mpm* h, float dt, int32_t n_substeps, const uint32_t* bc_active,
                               float* kernel_ms, void* stream);
/* Measurement: average duration (ms) of one launch of k_p2g, k_grid, k_g2p
 * and the binning, each launched `reps` times back to back between two
 * hipEvents on `stream` (so event overhead is amortised); the launches use the
 * current substep's inputs (BC mask `bc_active`).  Fused pipeline: {k_fused
 * (G2P + P2G), k_grid_f, binning, 0}.  Particle state and bins are
 * restored afterwards.  Synchronises `stream`. */
int gsmpm_mpm_time_kernels(gsmpm_mpm* h, float dt, uint32_t bc_active, int32_t reps, float* ms4, void* stream);
/* Diagnostics of the tile buckets the next substep reads: {active tiles, max
 * particles in a tile, particles outside the grid, chunks, touched tiles (owned
 * by the next grid update), binned total, parity, substeps since the last
 * re-sort}.  Synchronises `stream`. */
int gsmpm_mpm_debug_stats(gsmpm_mpm* h, int32_t* out8, void* stream);
/* Workgroup timelines of the last k_p2g / k_g2p / k_finish_bins launches:
 * out[4][8192][8] phase stamps in s_memrealtime ticks (100 MHz).  Diagnostics. */
int gsmpm_debug_stamps(uint64_t* out, void* stream);
/* Node box (lo[3], hi[3]) of the tiles the next grid update owns; synchronises `stream`. */
int gsmpm_mpm_live_box(gsmpm_mpm* h, int32_t* box6, void* stream);

/* Device 3x3 SVD (the ti.svd restatement used by the constitutive kernels) on
 * n row-major matrices: A[n*9] -> U[n*9], sig[n*3], V[n*9].  Test entry point. */
int gsmpm_svd3(const float* A, int32_t n, float* U, float* sig, float* V, void* stream);

/* Constitutive step alone (compute_stress_from_F_trial, utils.py:13-54) on n
 * particles: F_trial[n*9], mu[n], lam[n], yield[n] (updated in place for
 * metal) -> F[n*9] (return-mapped), tau[n*9] (symmetrised Kirchhoff stress).
 * material: GSMPM_MAT_*, or 4 = jelly with FCR (F3 fixed), or 5 = the cohesive
 * fluid of fluid_return_mapping (constitutive_models.py:142-213; defined but
 * never dispatched by the reference) with StVK stress.  Test entry point. */
int gsmpm_constitutive(int32_t material, const float* F_trial, int32_t n, const float* mu, const float* lam,
                       float* yield, float dt, float* F_out, float* tau_out, void* stream);

/* get_particle_volume (internel_filling/filling.py:27-42): vol[N] from
 * x[N,3] (grid space) with an n^3 i32 count grid in `scratch` (>= 4*n^3 B). */
int gsmpm_particle_volume(const float* x, int32_t n, int32_t n_grid, double grid_extent, int32_t* scratch,
                          float* vol_out, void* stream);

/* ------------------------------------------------ differentiable MPM ---
 * Replaces MPM_Simulator with args.fitting=True (solver.py:54-108,131-133,
 * 167-177) over MPM_model's logE/y/mu/lam (model.py:35-44) and
 * MPM_state_opt (model.py:135-223): L state levels of x, v, F, stress, C
 * (level s+1 = substep s of level s), adjoints of all of them, the dense grid
 * and its adjoints.  Same numerics and the same accumulation behaviour as
 * Taichi's reverse mode on those kernels.
 */
typedef struct gsmpm_fit gsmpm_fit;

typedef struct {
  int32_t n_particles;
  int32_t n_grid;               /* MPMParams.n_grid */
  double grid_extent;
  int32_t levels;               /* 31 in the reference (model.py:145-149) */
  double E, nu, density;        /* logE = log10 E, y = -log(0.49/nu - 1) (model.py:41-43) */
  double gravity[3];
} gsmpm_fit_params;

int gsmpm_fit_create(const gsmpm_fit_params* p, gsmpm_fit** out);
int gsmpm_fit_destroy(gsmpm_fit* h);
/* MPM_state_opt.__init__ + init2 (model.py:150-187): xyz [N,3], cov6 [N,6],
 * vol [N], init_v [N,3] (NULL = 0) as level 0; F[0] = I, C[0] = stress[0] = 0;
 * mass = density * vol; mu/lam from logE/y (model.py:44). */
int gsmpm_fit_set_particles(gsmpm_fit* h, const float* xyz, const float* cov6, const float* vol,
                            const float* init_v, void* stream);
/* grid_postprocess[0] as a fixed cube (set_bc_ground_only, solver.py:131-133,
 * StickyGroundBC boundary_conditions.py:88-95 = center (1,0.6,1), size (1,0.1,1)). */
int gsmpm_fit_set_fixed_cube(gsmpm_fit* h, const double center[3], const double size[3]);
/* p2g2p_forward(dt, s), solver.py:54-69: level s -> level s+1. */
int gsmpm_fit_forward(gsmpm_fit* h, float dt, int32_t s, void* stream);
/* p2g2p_backward(dt, s), solver.py:71-90. */
int gsmpm_fit_backward(gsmpm_fit* h, float dt, int32_t s, void* stream);
/* postprocess_forward / _backward, solver.py:167-171 (compute_cov_from_F_opt, utils.py:435-467) */
int gsmpm_fit_postprocess_forward(gsmpm_fit* h, void* stream);
int gsmpm_fit_postprocess_backward(gsmpm_fit* h, void* stream);
/* MPM_state_opt.set_grads (model.py:192-202): xyz_grad [N,3] -> x.grad[L-1], cov_grad [6N] -> cov.grad */
int gsmpm_fit_set_grads(gsmpm_fit* h, const float* xyz_grad, const float* cov_grad, void* stream);
int gsmpm_fit_learn(gsmpm_fit* h, void* stream);        /* solver.py:92-108 */
int gsmpm_fit_cycle_init(gsmpm_fit* h, void* stream);   /* model.py:216-223 */
int gsmpm_fit_clear_grads(gsmpm_fit* h, void* stream);  /* solver.py:173-175 */
int gsmpm_fit_mu_lam(gsmpm_fit* h, void* stream);       /* compute_mu_lam_from_E_nu, utils.py:349-362 */

/* Fields, external particle order; leveled ones take `level`, the rest ignore it. */
#define GSMPM_FIT_X 0          /* particle_xyz[level]    [N,3] */
#define GSMPM_FIT_V 1          /* particle_vel[level]    [N,3] */
#define GSMPM_FIT_F 2          /* particle_F[level]      [N,9] */
#define GSMPM_FIT_C 3          /* particle_C[level]      [N,9] */
#define GSMPM_FIT_STRESS 4     /* particle_stress[level] [N,9] */
#define GSMPM_FIT_GX 5         /* .grad of the above, same shapes */
#define GSMPM_FIT_GV 6
#define GSMPM_FIT_GF 7
#define GSMPM_FIT_GC 8
#define GSMPM_FIT_GSTRESS 9
#define GSMPM_FIT_LOGE 10      /* [N] */
#define GSMPM_FIT_Y 11
#define GSMPM_FIT_MU 12
#define GSMPM_FIT_LAM 13
#define GSMPM_FIT_GLOGE 14
#define GSMPM_FIT_GY 15
#define GSMPM_FIT_GMU 16
#define GSMPM_FIT_GLAM 17
#define GSMPM_FIT_COV 18       /* particle_cov [N,6] */
#define GSMPM_FIT_GCOV 19
#define GSMPM_FIT_INIT_COV 20
#define GSMPM_FIT_VOL 21
#define GSMPM_FIT_MASS 22
#define GSMPM_FIT_FIELD_COUNT 23
int gsmpm_fit_field_width(int32_t field);
int gsmpm_fit_get(gsmpm_fit* h, int32_t field, int32_t level, float* out, void* stream);
int gsmpm_fit_set(gsmpm_fit* h, int32_t field, int32_t level, const float* in, void* stream);
/* Dense grid of the last substep: GSMPM_GRID_MASS [n^3], _V_IN / _V_OUT [n^3,3],
 * and 3 / 4 for grid_v_in.grad / grid_v_out.grad [n^3,3]. */
int gsmpm_fit_get_grid(gsmpm_fit* h, int32_t which, float* out, void* stream);

/* -------------------------------------------------------- rasterizer ---
 * Replaces diff_gaussian_rasterization._C.rasterize_gaussians (forward;
 * called via GaussianRasterizer.forward at main.py:148-156).  Upstream
 * third-party, pre-2024 API; not vendored in the reference.
 */
typedef struct gsmpm_raster gsmpm_raster;

typedef struct {
  int32_t P;                 /* number of Gaussians */
  int32_t D;                 /* sh degree */
  int32_t M;                 /* SH coefficients per Gaussian (shs.size(1)), 0 if colors_precomp */
  int32_t W, H;
  const float* means3D;      /* [P,3] */
  const float* shs;          /* [P,M,3] or NULL */
  const float* colors_precomp; /* [P,3] or NULL */
  const float* opacities;    /* [P] */
  const float* scales;       /* [P,3] or NULL */
  const float* rotations;    /* [P,4] or NULL */
  const float* cov3D_precomp;/* [P,6] or NULL */
  float scale_modifier;
  const float* viewmatrix;   /* [4,4] (transposed world->view, as upstream) */
  const float* projmatrix;   /* [4,4] */
  const float* campos;       /* [3] */
  const float* bg;           /* [3] */
  float tanfovx, tanfovy;
  int32_t prefiltered;
} gsmpm_raster_args;

int gsmpm_raster_create(gsmpm_raster** out);
int gsmpm_raster_destroy(gsmpm_raster* r);
/* out_color [3,H,W] f32, out_radii [P] i32 (device).  *num_rendered gets K.
 * The binning buffers grow inside the context (not graph-capturable: the
 * upstream forward also syncs on num_rendered). */
int gsmpm_raster_forward(gsmpm_raster* r, const gsmpm_raster_args* a, float* out_color, int32_t* out_radii,
                         int32_t* num_rendered, void* stream);
/* Replaces _C.rasterize_gaussians_backward (upstream's _RasterizeGaussians.backward,
 * used by extra.py's loss.backward(), extra.py:198-200,218).  Uses the state of
 * the last gsmpm_raster_forward on this context (same args; keep one context
 * per differentiable forward).  dL_dcolor [3,H,W]; outputs, all [P,...] and
 * fully written: dL_dmeans2D [P,3] (w.r.t. NDC, z = 0), dL_dcolors [P,3],
 * dL_dopacity [P], dL_dmeans3D [P,3], dL_dcov3D [P,6], dL_dsh [P,M,3] (if
 * shs), dL_dscales [P,3] and dL_drotations [P,4] (if scales/rotations). */
int gsmpm_raster_backward(gsmpm_raster* r, const gsmpm_raster_args* a, const int32_t* radii, const float* dL_dcolor,
                          float* dL_dmeans2D, float* dL_dcolors, float* dL_dopacity, float* dL_dmeans3D,
                          float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations, void* stream);
/* Forward-only context (on != 0): gsmpm_raster_forward skips the per-pixel
 * state (final T, last contributor: 8 B a pixel) that only a backward reads,
 * and gsmpm_raster_backward on it fails.  Used for main.py's frames
 * (main.py:148-157 never differentiates); autograd forwards use contexts
 * with it off (the default). */
int gsmpm_raster_set_forward_only(gsmpm_raster* r, int32_t on);
/* Caller-owned workspace form of the forward (upstream's
 * RasterizeGaussiansCUDA takes torch byte tensors for its geometry / binning /
 * image buffers, rasterize_points.cu).  gsmpm_raster_workspace_size: the
 * bytes a forward of P Gaussians into an H x W image needs when the frame
 * bins at most `pairs` (Gaussian, tile) pairs (pairs = 0: the part that does
 * not depend on the pair count).  gsmpm_raster_forward_ws: the forward with
 * every buffer carved from `workspace` (device memory, 256-byte aligned,
 * ws_bytes long, ZERO-FILLED ONCE when created: the hand-written depth order
 * keeps its bucket state at the workspace's start and leaves it zero after
 * every call); no allocation inside, forward-only (no backward state).
 * The pair count is known only after the binning scan (upstream resizes its
 * binning buffer at that point): when the frame needs more pairs than the
 * workspace holds, the call returns GSMPM_ESPACE with *pairs_needed set,
 * out_color and num_rendered unwritten, and out_radii possibly overwritten
 * (k_preprocess runs before the count is known); the depth-order kernels may
 * still be queued on `stream` at return (they leave the workspace's state
 * zero), so the old workspace must not be freed for reuse by another stream
 * before `stream` reaches that point.  The caller sizes a larger workspace
 * for that many pairs and calls again. */
int gsmpm_raster_workspace_size(int32_t P, int32_t H, int32_t W, int64_t pairs, uint64_t* bytes);
int gsmpm_raster_forward_ws(const gsmpm_raster_args* a, float* out_color, int32_t* out_radii,
                            int32_t* num_rendered, void* workspace, uint64_t ws_bytes, int64_t* pairs_needed,
                            void* stream);
/* The forward with the pair count left on the device (the round-4 verdict's
 * item 4: upstream and gsmpm_raster_forward_ws read it on the host to size
 * the binning, main.py:148-156).  The pair buffers are carved for pairs_cap
 * pairs (the workspace must hold gsmpm_raster_workspace_size(P, H, W,
 * pairs_cap), else GSMPM_ESPACE before any launch); every launch size is
 * fixed by P, H, W and pairs_cap, the kernels cut at the device's count, and
 * nothing waits on the host: the call only enqueues on `stream`, and the
 * sequence can be captured into a graph and replayed (the argument pointers
 * are baked in).  When the stream reaches the end, counts (device-accessible:
 * host-mapped pinned or device memory, 4 words) holds {K, num_rendered,
 * flags, internal}: flags bit 0 = a depth bucket above 8,192 Gaussians (the hand-
 * written order needs its LSD fallback, which this form does not take), bit 1
 * = K > pairs_cap (the emission stopped at pairs_cap).  Either bit means
 * out_color is not the frame: render it again with gsmpm_raster_forward_ws
 * (or with pairs_cap >= K).  The default depth-ordered path with the chunked
 * tile sort only (<= 4,096 tiles: the lego camera's 2,500); more tiles or an
 * A/B switch that selects another path: GSMPM_EINVAL. */
int gsmpm_raster_forward_async(const gsmpm_raster_args* a, float* out_color, int32_t* out_radii, void* workspace,
                               uint64_t ws_bytes, int64_t pairs_cap, uint32_t* counts, void* stream);

/* In-frame timing of the forwards (diagnostics; process-wide).  With timing
 * on, every forward not issued into a stream capture records three events on
 * its stream (entry, before and after k_render); gsmpm_raster_timing waits
 * for the forwards recorded since the last call and returns the sums of
 * their k_render and whole-forward times (ms) and their count.  Replaces
 * nothing in the reference (upstream has no timing); bench.py reports
 * k_render's in-frame average with it. */
int gsmpm_raster_set_timing(int32_t on);
int gsmpm_raster_timing(double* k_render_ms, double* forward_ms, int64_t* forwards);
/* Diagnostics of the context's last forward: *binned = the (Gaussian, tile)
 * pairs actually sorted and listed (each Gaussian binned into the tiles its
 * alpha >= 1/255 box reaches, a subset of the 3-sigma rect), *rendered = its
 * num_rendered (upstream's 3-sigma pair count).  Either pointer may be null. */
int gsmpm_raster_pair_counts(const gsmpm_raster* r, uint32_t* binned, uint32_t* rendered);
/* Diagnostics of the context's last hand-written depth order (csrc/dsort.h):
 * out8 = {buckets, occupied buckets sorted by a wave, by a workgroup, largest
 * bucket, overflow flag, visible Gaussians, fallbacks so far (a bucket above
 * 8,192 entries: the LSD form instead), shift}. */
int gsmpm_raster_dsort_stats(const gsmpm_raster* r, int64_t out8[8]);
/* GaussianRasterizer.markVisible -> _C.mark_visible: visible[P] (u8) = view z > 0.2 */
int gsmpm_raster_mark_visible(const float* means3D, int32_t P, const float* viewmatrix, const float* projmatrix,
                              uint8_t* visible, void* stream);

#ifdef __cplusplus
}
#endif
#endif
