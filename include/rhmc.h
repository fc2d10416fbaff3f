/*
 * rhmc.h — C-ABI of the MI355X-native RHMC leapfrog engine (librhmc.so).
 *
 * Drop-in boundary for ONE hot path of jaekor91/HMC-stellar-toy-model: the
 * implicit generalized-leapfrog step of the Riemannian-HMC sampler for the
 * Poisson / Gaussian-PSF stellar-photometry posterior.
 *
 * Reference interface each entry point replaces (file:line into the
 * reference checkout):
 *   rhmc_leapfrog / rhmc_leapfrog_device
 *       base_class.RHMC_single_step(q, p, delta, counter_max)
 *       sampler_RHMC.py:522-566, called Nsteps times per MH iteration from
 *       multi_gym.run_RHMC (sampler_RHMC.py:1053-1054) and inlined in
 *       single_gym.run_single_RHMC solver="implicit" (:729-772).
 *       n_steps consecutive steps are fused into one launch.
 *   rhmc_gradient
 *       base_class.dVdq (sampler_RHMC.py:365-425) and base_class.dphidq
 *       (:448-465), batched over chains.
 *   rhmc_energy / rhmc_energy_device
 *       base_class.V (sampler_RHMC.py:294-351) and base_class.T (:353-363)
 *       at H(q) (:229-258) — the trajectory-endpoint energies of the MH test
 *       (:1021-1026, :1070-1071).
 *   rhmc_mh / rhmc_mh_device
 *       multi_gym.run_RHMC, move-0 ("within") branch (sampler_RHMC.py:1018-1083):
 *       momentum draw p = z*sqrt(H(q)) (:1021-1022), E0 = V + T (:1025-1027),
 *       Nsteps leapfrog steps (:1053-1054), E1, accept if dE < 0 or
 *       ln u < -dE (:1072-1083) — n_iter iterations, all on the device.
 *       rhmc_mh_scheduled(_device): the same with run_RHMC's schedule_g_ff2 /
 *       schedule_beta (:1010-1016).
 *   rhmc_integrate / rhmc_integrate_device
 *       the reference's other integrators, selected by RHMC_SOLVER_*:
 *       single_gym.run_single_HMC leapfrog (sampler_RHMC.py:628-645) and
 *       single_gym.run_single_RHMC solver="naive" (:690-708) / "leap_frog"
 *       (:709-728); RHMC_SOLVER_IMPLICIT is RHMC_single_step.
 *   rhmc_ctx_create / rhmc_ctx_set_image
 *       the instance attribute base_class.D set by gen_mock_data
 *       (sampler_RHMC.py:77-99); uploaded once per context.
 *   rhmc_gen_image / rhmc_gen_image_device
 *       base_class.gen_model (sampler_RHMC.py:101-116), gen_mock_data
 *       (:77-99, Poisson draw utils.py:488-496) and the N_trial realisations
 *       of gen_noise_profile (:118-144), on the device.
 *   rhmc_leapfrog_ragged_device / rhmc_energy_ragged_device /
 *   rhmc_rows_copy_device / rhmc_kinetic_rows_device (ABI 4)
 *       the same step and V for chains of DIFFERENT star counts in one launch,
 *       and the momentum draw / T of run_RHMC (:1021-1026, :353-363) on
 *       device-resident ragged sets: the reversible-jump iterations of
 *       run_RHMC (:1018-1187), whose chains change K by births, deaths,
 *       splits and merges (librhmc_rj.so keeps them in HBM between phases).
 *   rhmc_params
 *       the instance attributes the step reads: dt, g_xx,
 *       g_ff, g_ff2, g0, g1, g2, B_count, f_lim, mB (-> f_low),
 *       PSF_FWHM_pix, use_prior, alpha, use_Vc, beta, Vc_r_pow, plus the
 *       run_RHMC arguments delta / counter_max (:937-939).
 *
 * Conventions
 *   - Arrays are C-contiguous fp64 [n_chains][3K] with (f_k, x_k, y_k)
 *     interleaved per star, flux in counts (format_q, sampler_RHMC.py:209).
 *     D is fp64 [rows][cols], rows == cols (reference limitation:
 *     gauss_PSF returns (cols, rows), utils.py:481-483).
 *   - Host-pointer entry points are synchronous and update q, p in place.
 *     The *_device entry points take device pointers and a hipStream_t
 *     (passed as void*, NULL = the context's stream) and are asynchronous.
 *   - Every call returns 0 on success or a negative RHMC_ERR_* code;
 *     rhmc_last_error() gives a thread-local message.  No C++ exception
 *     crosses the ABI.  A context must not be used by two threads at once,
 *     except that rhmc_leapfrog_device, rhmc_energy_device,
 *     rhmc_leapfrog_ragged_device, rhmc_energy_ragged_device,
 *     rhmc_rows_copy_device, rhmc_kinetic_rows_device and rhmc_ragged_ok
 *     (which read the context's options and image and otherwise touch only a
 *     per-stream, mutex-guarded table buffer) may be called from several
 *     threads at once, on the same or distinct streams: a launch holds a
 *     reference to the table buffer it was given until it is enqueued, so a
 *     buffer grown by another thread is released only after that launch (the
 *     order of two threads' launches on one stream is theirs to arrange).
 *     Options must not change while such calls run.  One context per GPU.
 */
#ifndef RHMC_H
#define RHMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RHMC_ABI_VERSION 4

enum {
  RHMC_OK = 0,
  RHMC_ERR_ARG = -1,         /* bad argument (shape, NULL, K range ...) */
  RHMC_ERR_HIP = -2,         /* a HIP runtime call failed                */
  RHMC_ERR_NOMEM = -3,       /* device allocation failed                 */
  RHMC_ERR_UNSUPPORTED = -4  /* configuration not built into this library */
};

/* Integrators selectable through rhmc_integrate. */
enum {
  RHMC_SOLVER_IMPLICIT = 0,       /* RHMC_single_step (:522-566)                  */
  RHMC_SOLVER_HMC = 1,            /* plain leapfrog, unit metric (:628-645)       */
  RHMC_SOLVER_RHMC_NAIVE = 2,     /* explicit RHMC, "naive" (:690-708)            */
  RHMC_SOLVER_RHMC_LEAPFROG = 3   /* explicit RHMC, "leap_frog" (:709-728)        */
};

/* Per-chain status bits written by rhmc_leapfrog (OR over all steps). */
#define RHMC_STATUS_NONFINITE   1u  /* q or p became NaN/inf                    */
#define RHMC_STATUS_PLOOP_CAP   2u  /* p fixed-point loop stopped at counter_max */
#define RHMC_STATUS_QLOOP_CAP   4u  /* q fixed-point loop stopped at counter_max */
#define RHMC_STATUS_REFLECT_F   8u  /* flux-wall reflection (:558-559)           */
#define RHMC_STATUS_REFLECT_XY 16u  /* edge reflection (:561-564)                */
/* A reflection of the implicit step fired with its coordinate within 2^-40 (9.1e-13) of
 * the wall (relative to max(1, |wall|): f_lim, 0 or R-1; :554-564).  Such a
 * chain can legitimately reflect the other way on a last-bit difference
 * (SURVEY §8(c)), so callers report these chains separately. */
#define RHMC_STATUS_NEAR_WALL  32u

/* Instance state read by the step (POD; all fp64 except the flags). */
typedef struct rhmc_params {
  double dt;           /* self.dt                                            */
  double delta;        /* fixed-point tolerance (absolute, max-norm)         */
  double B_count;      /* background counts per pixel                        */
  double f_lim;        /* flux wall (counts)                                 */
  double f_low;        /* H_xx clamp = mag2flux(mB+2)*flux_to_count (:267)   */
  double fwhm_pix;     /* PSF FWHM in pixels                                 */
  double g_xx, g_ff, g_ff2;
  double g0, g1, g2;   /* metric factors (utils.factors at 48x48, :165)      */
  double alpha;        /* prior exponent (used when use_prior)               */
  double beta;         /* repulsion strength (used when use_Vc)              */
  double Vc_r_pow;     /* repulsion power                                    */
  double V_prior_const;/* rhmc_energy only: the cached prior constant (:321) */
  int32_t counter_max; /* fixed-point iteration cap                          */
  int32_t use_prior;
  int32_t use_Vc;
  int32_t reserved;    /* must be 0                                          */
} rhmc_params;

typedef struct rhmc_ctx rhmc_ctx;

/*
 * Context options (rhmc_ctx_set_option).  Nothing in the library reads the
 * environment: kernel selection is per context, AUTO unless a caller (the
 * parity tests) sets it.
 *
 * RHMC_OPT_KERNEL: the kernel family the compute calls use.  A family that
 * does not serve the call's configuration (K, image side, PSF width, fp32
 * exactness of the image) leaves the automatic choice for that call.
 *   AUTO            the default dispatch
 *   GENERIC         one wave per chain, image in LDS (K <= 16, image + tables
 *                   fit LDS; else WINDOWED); explicit integrators and
 *                   HMC_random take WINDOWED; MH runs the four-kernel loop
 *   WINDOWED        one wave per chain, 32-px star windows, image in HBM/L2
 *   REGWIN          K = 1 register-window kernel at every batch size
 *   REGWIN32        ... forced onto the 32-px window
 *   REGWIN_F64      ... with an fp64 pixel cache
 *   LANE1 / LANE4   K = 1 lane-group kernel, 1 / 4 lanes per chain, at every
 *                   batch size; LANE1_F64: fp64 image in LDS
 *   PIXMAJOR        2 <= K <= 10 pixel-major kernel (the AUTO choice there)
 *   MULTIWIN        K >= 2 multi-star register-window kernel (also where the
 *                   pixel-major kernel would serve); MULTIWIN_NOTAB without
 *                   the LDS factor tables
 *   DENSE           the many-star kernel for 32/48-px images (full-image
 *                   pixel-major Lambda, star-major sums; the AUTO choice there
 *                   from 11 stars) at any K
 * RHMC_OPT_MH_FUSED: 1 (default) = one-launch MH where a fused kernel exists,
 *   0 = the four-kernel loop (begin / leapfrog / energy / end) always.
 * RHMC_OPT_WINDOW_SPLIT: waves per chain pair in the multi-star
 *   register-window kernel's implicit step (leapfrog_kr): 0 (default) = by
 *   batch size (1 from 2 waves per SIMD up, else 2 or 4, so that e.g. C5's
 *   8192 chains split over 8 GPUs still fill each one), or 1, 2, 4.  The
 *   results do not depend on it (bit-identical).  It applies only where that
 *   kernel runs the implicit step without LDS factor tables (images larger
 *   than 64 px, or K > 16); the factor-table variant, the explicit solvers,
 *   HMC_random and every other kernel family ignore it, and
 *   rhmc_ctx_get_option returns the value set either way.
 * RHMC_OPT_TABLES (diagnostic; results do not depend on it): the windowed
 *   kernels from 65 stars keep their per-chain PSF factor tables in global
 *   memory, one buffer per (context, stream).  STREAM (default) = that
 *   buffer; STREAM_POISON = the same, filled with 0xFF bytes (NaN) before
 *   every launch, so that a read of an entry the launch did not write would
 *   show as a NaN result (tests/test_gpu_tables_determinism.py: none does).
 *   The POOL* values (a stream-ordered pool allocation per launch, round 5's
 *   first scheme, and its variants) reproduce a defect outside the kernels
 *   (a reused pool block is zeroed while the launch that
 *   received it runs); only -DRHMC_TABLE_DIAG builds accept them, the library
 *   returns RHMC_ERR_UNSUPPORTED.
 */
enum {
  RHMC_OPT_KERNEL = 1,
  RHMC_OPT_MH_FUSED = 2,
  RHMC_OPT_WINDOW_SPLIT = 3,
  RHMC_OPT_TABLES = 4
};
enum {
  RHMC_TABLES_STREAM = 0,
  RHMC_TABLES_STREAM_POISON = 1,
  RHMC_TABLES_POOL = 2,
  RHMC_TABLES_POOL_POISON = 3,
  RHMC_TABLES_POOL_KEEP = 4,
  RHMC_TABLES_POOL_SYNCFREE = 5,
  RHMC_TABLES_POOL_BARRIER = 6
};
enum {
  RHMC_KERNEL_AUTO = 0,
  RHMC_KERNEL_GENERIC = 1,
  RHMC_KERNEL_WINDOWED = 2,
  RHMC_KERNEL_REGWIN = 3,
  RHMC_KERNEL_REGWIN32 = 4,
  RHMC_KERNEL_REGWIN_F64 = 5,
  RHMC_KERNEL_LANE1 = 6,
  RHMC_KERNEL_LANE4 = 7,
  RHMC_KERNEL_LANE1_F64 = 8,
  RHMC_KERNEL_PIXMAJOR = 9,
  RHMC_KERNEL_MULTIWIN = 10,
  RHMC_KERNEL_MULTIWIN_NOTAB = 11,
  RHMC_KERNEL_DENSE = 12
};
int rhmc_ctx_set_option(rhmc_ctx* ctx, int32_t option, int32_t value);
int rhmc_ctx_get_option(rhmc_ctx* ctx, int32_t option, int32_t* value);

/* ABI version of the loaded library (== RHMC_ABI_VERSION when in sync). */
int rhmc_abi_version(void);
/* Number of visible GPUs; 0 (and RHMC_OK) when none. */
int rhmc_device_count(int* n);
/* Thread-local message of the last failing call ("" if none). */
const char* rhmc_last_error(void);

/* Create a context on `device` and upload D [rows][cols] (host pointer). */
int rhmc_ctx_create(int device, const double* D, int32_t rows, int32_t cols,
                    rhmc_ctx** out);
/* Replace the data image (host pointer); may change the size. */
int rhmc_ctx_set_image(rhmc_ctx* ctx, const double* D, int32_t rows, int32_t cols);
/* Device pointer of the context's image (for callers that keep state on device). */
int rhmc_ctx_image_device(rhmc_ctx* ctx, const double** d_image);
void rhmc_ctx_destroy(rhmc_ctx* ctx);
/* Wait for all work queued on the context's stream. */
int rhmc_ctx_synchronize(rhmc_ctx* ctx);

/*
 * n_steps RHMC_single_step()s on every chain.  q, p: host [n_chains][3K],
 * updated in place.  fp_iters (nullable): host int32 [n_chains][2], the
 * p- and q-loop iteration counts summed over the n_steps steps.  status
 * (nullable): host int32 [n_chains], RHMC_STATUS_* bits.  1 <= K <= 1024 on
 * every step, gradient, energy and MH entry point (else RHMC_ERR_ARG).  From
 * 65 stars the windowed one-wave-per-chain kernels (images other than the
 * dense kernel's 32/48 px, or K > 256) keep their PSF factor tables in global
 * memory, 2 x 33 doubles per star per chain in a buffer the context keeps
 * per stream until rhmc_ctx_destroy (grown on demand after a sync of that
 * stream; RHMC_ERR_NOMEM if that fails); they need a PSF narrow
 * enough for the 32-pixel window (else RHMC_ERR_UNSUPPORTED).
 */
int rhmc_leapfrog(rhmc_ctx* ctx, const rhmc_params* P, double* q, double* p,
                  int64_t n_chains, int32_t K, int32_t n_steps,
                  int32_t* fp_iters, int32_t* status);

/* Same on device-resident buffers, asynchronous on `stream` (hipStream_t). */
int rhmc_leapfrog_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q,
                         double* d_p, int64_t n_chains, int32_t K,
                         int32_t n_steps, int32_t* d_fp_iters,
                         int32_t* d_status, void* stream);

/*
 * Ragged chain sets (ABI 4).  Chain i of a call is row rows[i] (d_rows NULL:
 * row i) of padded device arrays [*][ld]; the row holds the chain's d_K[row]
 * stars (its first 3 K entries; d_K indexed by row).  One launch serves every
 * star count in [K_min, K_max] when the automatic dispatch runs a slotted
 * one-wave-per-chain kernel for each of them — the dense kernel on 32/48-px
 * images from 11 stars, the windowed kernel — or the pixel-major kernel (2-10
 * stars on 32/48-px images whose pixels are exact in fp32; a launch takes one
 * family: 2-10 and 11+ stars are separate sets) (rhmc_ragged_ok says which K);
 * K_min and K_max must need the same register slots (1-64, 65-128, 129-256,
 * 257-512, 513-1024 stars), else RHMC_ERR_ARG, and a K the slotted kernels do not serve gives
 * RHMC_ERR_UNSUPPORTED.  Each chain's results equal those of a fixed-K call
 * on it (the kernels are batch-invariant).  Asynchronous on `stream`.
 */
int rhmc_ragged_ok(rhmc_ctx* ctx, const rhmc_params* P, int32_t K, int32_t* ok);
/* n_steps RHMC_single_step()s on the set; q, p rows updated in place. */
int rhmc_leapfrog_ragged_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, double* d_p,
                                int64_t ld, const int64_t* d_rows, const int32_t* d_K,
                                int64_t n, int32_t K_min, int32_t K_max, int32_t n_steps,
                                void* stream);
/* V (rhmc_energy's, f_pos bits likewise) of the set: d_V[i] for chain i. */
int rhmc_energy_ragged_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, int64_t ld,
                              const int64_t* d_rows, const int32_t* d_K, int64_t n,
                              int32_t K_min, int32_t K_max, int32_t f_pos, double* d_V,
                              void* stream);
/* dst[dst_rows[i]][0:width] = src[src_rows[i]][0:width] for i < n (either
 * index array NULL: row i): gathers of a ragged set into packed [n][3K]
 * batches for the fixed-K entry points, scatters back, row restores. */
int rhmc_rows_copy_device(rhmc_ctx* ctx, const double* d_src, int64_t ld_src,
                          const int64_t* d_src_rows, double* d_dst, int64_t ld_dst,
                          const int64_t* d_dst_rows, int64_t n, int32_t width, void* stream);
/* Rows 0..n-1 of a ragged set (d_K[c] stars): with d_z non-NULL first the
 * momentum draw p = z sqrt(H(q)) (:1021-1022; chain c's 3 K normals at
 * d_z + d_zoff[c], p zeroed past 3 K), then T[c] = (sum p^2/H(q) + sum
 * ln|H(q)|) / 2 (:353-363) with NumPy's pairwise summation order.  H
 * follows the reference's operation order (:260-292, g_ff2 / g_xx / B /
 * f_low from P).  1 <= d_K[c] <= 1024 (a larger count gets T = NaN). */
int rhmc_kinetic_rows_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, double* d_p,
                             int64_t ld, const int32_t* d_K, const double* d_z,
                             const int64_t* d_zoff, int64_t n, double* d_T, void* stream);

/* kind: 0 = dVdq (:365-425), 1 = dphidq (:448-465).  Host pointers. */
int rhmc_gradient(rhmc_ctx* ctx, const rhmc_params* P, const double* q,
                  double* grad, int64_t n_chains, int32_t K, int32_t kind);

/* V (:294-351) and T at H(q) (:353-363) per chain.  V or T may be NULL.  p
 * may be NULL when T is NULL.  Host pointers.  f_pos is a bit set:
 * RHMC_V_FLUX_WALL (1) = V is inf when a flux is below f_lim (:303-309, the
 * reference's f_pos=True); RHMC_V_NO_POSCHECK (2) = skip the position support
 * check (:311-317), i.e. samplers.lightsource_gym.V (samplers.py:1137-1150),
 * which has none. */
#define RHMC_V_FLUX_WALL   1
#define RHMC_V_NO_POSCHECK 2
int rhmc_energy(rhmc_ctx* ctx, const rhmc_params* P, const double* q,
                const double* p, double* V, double* T, int64_t n_chains,
                int32_t K, int32_t f_pos);
/* Same on device-resident buffers (d_V or d_T may be NULL; d_p may be NULL
 * when d_T is), asynchronous on `stream` (hipStream_t; NULL = the context's
 * stream).  Launches on distinct streams may run concurrently. */
int rhmc_energy_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q,
                       const double* d_p, double* d_V, double* d_T, int64_t n_chains,
                       int32_t K, int32_t f_pos, void* stream);

/* n_steps steps of integrator `solver` (RHMC_SOLVER_*) on every chain; q, p
 * host [n_chains][3K], updated in place.  f_pos: the flux-wall momentum flip of
 * the explicit RHMC solvers (:698-705, :719-726).  status nullable. */
int rhmc_integrate(rhmc_ctx* ctx, const rhmc_params* P, int32_t solver, double* q, double* p,
                   int64_t n_chains, int32_t K, int32_t n_steps, int32_t f_pos,
                   int32_t* status);
int rhmc_integrate_device(rhmc_ctx* ctx, const rhmc_params* P, int32_t solver, double* d_q,
                          double* d_p, int64_t n_chains, int32_t K, int32_t n_steps,
                          int32_t f_pos, int32_t* d_status, void* stream);

/* samplers.lightsource_gym.HMC_random's trajectory (samplers.py:519-552;
 * the MH bookkeeping around it, :489-568, stays on the host): unit-mass
 * leapfrog with the per-coordinate step vector dt[3K] (the reference's
 * self.dt) and steps[c] >= 1 steps for chain c (its np.random.randint draw),
 * flux wall at P->f_lim with the reference's quirks (sticky flip mask; when
 * the last step flipped, p is left at its input value and the chain's status
 * gets RHMC_STATUS_REFLECT_F).  q, p host [n_chains][3K] updated in place;
 * status nullable.  Gradient: dVdq without metric (:1108-1135). */
int rhmc_hmc_random(rhmc_ctx* ctx, const rhmc_params* P, const double* dt, double* q, double* p,
                    const int32_t* steps, int64_t n_chains, int32_t K, int32_t* status);
int rhmc_hmc_random_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_dt,
                           double* d_q, double* d_p, const int32_t* d_steps, int64_t n_chains,
                           int32_t K, int32_t* d_status, void* stream);

/* Per-iteration records of rhmc_mh (all nullable; host pointers for rhmc_mh,
 * device pointers for rhmc_mh_device).  Row l holds the state at the START
 * of iteration l, like the reference's q_chain / E_chain / V_chain / T_chain
 * (:1038-1042); accept[l] is A_chain[l] (:1077). */
typedef struct rhmc_mh_record {
  double* q_chain;   /* [n_iter][n_chains][3K] */
  double* E_chain;   /* [n_iter][n_chains] */
  double* V_chain;   /* [n_iter][n_chains] */
  double* T_chain;   /* [n_iter][n_chains] */
  int32_t* accept;   /* [n_iter][n_chains] */
} rhmc_mh_record;

/*
 * n_iter MH iterations of n_steps leapfrog steps each on every chain; q
 * [n_chains][3K] is updated in place to the last accepted state.  Randoms:
 * z [n_iter][n_chains][3K] standard normals and u [n_iter][n_chains] uniforms
 * in (0,1] — pass the reference's own NumPy draws for bit-level parity of the
 * accept sequence; NULL draws them on the device (Philox-4x32-10, `seed`,
 * counter = (index, iteration, chain)).  P->V_prior_const must be set when
 * use_prior.
 */
int rhmc_mh(rhmc_ctx* ctx, const rhmc_params* P, double* q, int64_t n_chains, int32_t K,
            int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* z, const double* u,
            uint64_t seed, const rhmc_mh_record* rec);
int rhmc_mh_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, int64_t n_chains,
                   int32_t K, int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* d_z,
                   const double* d_u, uint64_t seed, const rhmc_mh_record* rec, void* stream);

/*
 * Parameter schedules of multi_gym.run_RHMC (schedule_g_ff2 / schedule_beta,
 * sampler_RHMC.py:937-939, :1010-1016; RHMC-big-sim3.py:11-12): MH iteration
 * l of the call runs with g_ff2 = g_ff2[l] and beta = beta[l] while l < the
 * array's size, and with its last value after it; a NULL array (size 0)
 * keeps P's value.  Host arrays, for the device entry point too (they set
 * each iteration's constants).  P->g_ff2 / P->beta are not modified.
 */
typedef struct rhmc_mh_schedule {
  const double* g_ff2;  /* [n_g_ff2] or NULL */
  const double* beta;   /* [n_beta] or NULL  */
  int32_t n_g_ff2;
  int32_t n_beta;
} rhmc_mh_schedule;
/* rhmc_mh / rhmc_mh_device with a schedule (sched NULL: identical to them). */
int rhmc_mh_scheduled(rhmc_ctx* ctx, const rhmc_params* P, double* q, int64_t n_chains,
                      int32_t K, int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* z,
                      const double* u, uint64_t seed, const rhmc_mh_record* rec,
                      const rhmc_mh_schedule* sched);
int rhmc_mh_scheduled_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q,
                             int64_t n_chains, int32_t K, int32_t n_iter, int32_t n_steps,
                             int32_t f_pos, const double* d_z, const double* d_u, uint64_t seed,
                             const rhmc_mh_record* rec, const rhmc_mh_schedule* sched,
                             void* stream);

/*
 * Data generation.  q: [K][3] (flux in counts, x, y), K >= 0.  n_real == 0:
 * the model image B_count + sum_k f_k PSF_k (gen_model, sampler_RHMC.py:101-116;
 * per pixel exp(-((i+.5-x)^2 + (j+.5-y)^2) / (2 sigma^2)) / (2 pi sigma^2),
 * utils.py:475-486) into out [rows][cols].  n_real >= 1: n_real independent
 * Poisson realisations of it (gen_mock_data :77-99 / gen_noise_profile
 * :130-133) into out [n_real][rows][cols]; the Poisson sampler is NumPy's
 * legacy algorithm (multiplication below lam 10, PTRS above) on Philox-4x32-10
 * keyed by `seed` and the pixel index — the same distribution as the
 * reference, not the same stream.  Only P->B_count and P->fwhm_pix are read
 * (P->reserved must be 0).  install != 0 makes image 0 the context's data
 * image without a host round trip (rows == cols); out may then be NULL.
 * rhmc_ctx_create accepts D == NULL for a context that gets its image here.
 */
int rhmc_gen_image(rhmc_ctx* ctx, const rhmc_params* P, const double* q, int32_t K,
                   int32_t rows, int32_t cols, int32_t n_real, uint64_t seed, double* out,
                   int32_t install);
/* Device pointers, asynchronous on `stream`; d_out [max(n_real,1)][rows][cols]. */
int rhmc_gen_image_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, int32_t K,
                          int32_t rows, int32_t cols, int32_t n_real, uint64_t seed,
                          double* d_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RHMC_H */
