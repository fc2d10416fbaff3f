/*
 * rhmc_rj.h — C-ABI of librhmc_rj.so: the reversible-jump MCMC driver of the
 * reference, multi_gym.run_RHMC with P_move[1:] != 0 (sampler_RHMC.py:937-1198;
 * birth_death_move :1200-1270, split_merge_move :1273-1445), run natively for
 * many independent chains at once around the engine of rhmc.h.
 *
 * Chain c is run_RHMC after np.random.seed(seeds[c]): its random numbers come
 * from its own replica of NumPy's legacy RandomState (MT19937 with the legacy
 * normal / gamma / beta / bounded-integer algorithms), drawn in the
 * reference's order — momentum randn(3K) (:1021-1022), the move-type choice
 * (:1045), the grow/shrink choice (:1094, :1140), the move's own draws
 * (:1219-1221, :1231, :1249, :1291, :1300-1302, :1328, :1333, :1415) and the
 * accept uniform (:1075, :1164) — so the draws are the reference's bit for
 * bit.
 *
 * rhmc_rj_run keeps the chains in HBM for the whole run (round 5): every
 * chain's state, iteration-start state and momentum are rows of padded
 * [n][3 N_max] device arrays, and per iteration only the host-drawn normals,
 * a few doubles per chain (T, V), the jumping chains' rows (their proposals
 * run on the host, on a pool of host threads) and — when recorded — the
 * q_chain / p_chain rows cross PCIe.  The momentum p = z sqrt(H(q)) and both
 * kinetic energies run on the device (rhmc_kinetic_rows_device); every phase
 * is one ragged launch per register-slot class for the star counts the
 * slotted kernels serve (rhmc_leapfrog_ragged_device /
 * rhmc_energy_ragged_device: the dense kernel from 11 stars on 32/48-px
 * images, the windowed kernel) plus one packed launch per other star count
 * (gathered by rhmc_rows_copy_device).  The engine's results do not depend on
 * the batch a chain is in, so the records equal those of one run_RHMC per
 * seed.  rhmc_rj_run_physics runs the same iteration on host arrays around
 * caller-supplied engine callbacks (stand-ins for tests), one call per
 * distinct star count and phase.
 *
 * Concurrency: each pipe of a run uses device buffers and two HIP streams of
 * its own, held (a mutex) for the whole run, so concurrent rhmc_rj_run calls
 * on one device serialise pipe by pipe; the caller's current device is
 * restored on return.  The pipes' host work runs on one process-wide thread
 * pool per size (n_threads - pipes workers, kept for the process's lifetime,
 * shared by concurrent runs); the pipe threads take its chunks while their
 * streams run.  Host <-> device data moves through coherent pinned host
 * memory mapped into the device (the engine's kernels read and write it at
 * its device address): no copy-engine transfers.
 *
 * Retention: those buffers and the chains' host state (per device and pipe
 * index, grown to the largest run so far: ~90 MB of HBM and ~60 MB of pinned
 * host memory per pipe at 4,096 chains and N_max 120, 8 pipes from 16,384
 * chains) stay allocated after a run, so the next run starts without
 * allocating;
 * rhmc_rj_release(device) frees them (device < 0: every device), waiting for
 * a run that holds one.
 *
 * Replaces: the per-chain Python loop of run_RHMC's reversible-jump branches
 * (one chain, one star count at a time) — this is its batched, native form.
 *
 * Where the reference itself cannot continue (a death or merge that would
 * leave no star, a birth or split beyond N_max, a merge whose pair
 * probabilities are all zero — the reference raises there), the proposal is
 * rejected: the chain returns to the iteration's starting state, the rest of
 * the move's draws and the accept uniform are not drawn, and the iteration's
 * record gets RHMC_RJ_DEAD_END in `flags`.
 *
 * Arithmetic: the random draws are bit-identical to NumPy's; the metric and
 * kinetic-energy expressions follow the reference's operation order, with
 * C libm log/exp where NumPy may use its own SIMD versions (a last-bit
 * difference is possible there; tests/test_rj_native_host.py bounds it).
 *
 * Errors: 0 or a negative RHMC_ERR_* code (rhmc.h); rhmc_rj_last_error()
 * gives a thread-local message (an engine failure copies the engine's
 * last-error message).
 */
#ifndef RHMC_RJ_H
#define RHMC_RJ_H

#include <stdint.h>

#include "rhmc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The engine work of a run: the energy V(q) (rhmc_energy's V, f_pos bits) of
 * n chains of K stars, and n_steps RHMC_single_step()s on them (rhmc_leapfrog,
 * q and p updated in place).  Host arrays [n][3K].  Return 0 or a negative
 * code.  rhmc_rj_run wires them to a context; rhmc_rj_run_physics takes any
 * implementation (tests use stand-ins; the call order is deterministic). */
typedef struct rhmc_rj_physics {
  void* user;
  int (*energy)(void* user, const rhmc_params* P, const double* q, int64_t n, int32_t K,
                int32_t f_pos, double* V);
  int (*steps)(void* user, const rhmc_params* P, double* q, double* p, int64_t n, int32_t K,
               int32_t n_steps);
} rhmc_rj_physics;

/* One chain's NumPy legacy stream: RandomState.get_state() = ('MT19937', key,
 * pos, has_gauss, cached_gaussian).  2512 bytes. */
typedef struct rhmc_np_state {
  uint32_t key[624];
  int32_t pos;
  int32_t has_gauss;
  double gauss;
} rhmc_np_state;

typedef struct rhmc_rj_config {
  int32_t n_iter;        /* Niter: iterations 0 .. n_iter (n_iter + 1 records)      */
  int32_t n_steps;       /* Nsteps per trajectory                                    */
  int32_t N_max;         /* record width 3 N_max; star counts stay in [1, N_max]     */
  int32_t f_pos;         /* V's f_pos bits (RHMC_V_FLUX_WALL = run_RHMC f_pos=True)  */
  int32_t rows, cols;    /* num_rows / num_cols (birth positions, :1219-1220)       */
  int32_t n_threads;     /* host threads, the pipe threads included; <= 0:
                            min(hardware threads, 16)                             */
  int32_t n_g_ff2;       /* schedule_g_ff2 length (0: none)                          */
  int32_t n_beta;        /* schedule_beta length (0: none)                           */
  int32_t n_pipes;       /* 1: one pass over all chains per phase; 2..8: the chains in
                            that many contiguous parts on as many host threads, so
                            one part's host work overlaps the others' GPU work; 0:
                            2 from 1,024 chains, 3 from 2,048, 4 from 4,096, 8 from
                            16,384                                                    */
  int32_t use_states;    /* 1: the chains' streams start from states[c] instead of
                            seeds[c] (a checkpoint of an earlier run, or any
                            RandomState's get_state(): continue its stream)        */
  int32_t records_zero_padded; /* bits (0: none; was `reserved`), claims about the
                            caller's buffers that let the driver write a row's
                            zeros only up to its old width.  RHMC_RJ_ZP_RECORDS:
                            the q_chain / p_chain rows are zero past 3 n_stars[r]
                            on entry, n_stars holding the counts of the rows they
                            hold (a previous run's records of this shape, or
                            zeros: then any width is claimed; needs
                            rec->n_stars).  RHMC_RJ_ZP_STARTS: q's rows are
                            zero past 3 K[c] on entry (rhmc_rj_pack_starts
                            leaves them so)                                      */
  double P_move[3];      /* within / birth-death / split-merge probabilities         */
  double fmin, fmax;     /* power-law flux prior range, counts (:1221)               */
  double K_split;        /* split offset scale (:1300)                               */
  double beta_a, beta_b; /* split fraction F ~ Beta(beta_a, beta_b) (:1302)          */
  const double* schedule_g_ff2;  /* iteration l: g_ff2 = s[min(l, n - 1)] (:1010-1013) */
  const double* schedule_beta;   /* likewise beta (:1014-1016)                        */
  rhmc_np_state* states;         /* nullable [n]: read when use_states, and written with
                                    every chain's stream at the end of the run (resume a
                                    run from its q, K and states: the same draws as one
                                    uninterrupted run)                                 */
} rhmc_rj_config;

/* Per-iteration records, row l = the state at the START of iteration l
 * (run_RHMC's q_chain / p_chain / E_chain / V_chain / T_chain / N_chain /
 * move_chain / A_chain, :980-1003), iteration-major.  All nullable. */
typedef struct rhmc_rj_record {
  double* q_chain;   /* [n_iter+1][n][3 N_max], zero past the chain's 3K */
  double* p_chain;   /* [n_iter+1][n][3 N_max]                            */
  double* E_chain;   /* [n_iter+1][n]                                     */
  double* V_chain;
  double* T_chain;
  int32_t* accept;   /* A_chain                                           */
  int32_t* move;     /* 0 within, 1 birth, 2 death, 3 split, 4 merge      */
  int32_t* n_stars;  /* N_chain                                           */
  int32_t* flags;    /* RHMC_RJ_* bits of the iteration                   */
  double* phase_s;   /* [7] wall seconds summed over the run (and over the
                        pipes): momentum + move draws (host), V(q), first
                        trajectories, proposals (host), second
                        trajectories, V(q'), accept (host).  rhmc_rj_run
                        overlaps device and host work, so its phases are
                        the host's waits: [1] only queueing the momentum,
                        T, V(q) and the first trajectories, [2] their
                        completion, [4] queueing the second ones, [5]
                        their completion with V(q') and T', [6] the
                        iteration's record rows and the accept step        */
} rhmc_rj_record;

#define RHMC_RJ_DEAD_END 1u  /* the proposal could not be formed; rejected */
#define RHMC_RJ_ZP_RECORDS 1  /* rhmc_rj_config::records_zero_padded bits */
#define RHMC_RJ_ZP_STARTS 2

/*
 * Run n_iter + 1 iterations on n chains.  q: host [n][3 N_max], chain c's
 * first 3 K[c] entries (flux in counts, x, y per star; format_q); K: [n]
 * star counts, 1 <= K[c] <= N_max <= 1024.  Both are updated in place to the
 * chains' final states.  seeds: [n] (np.random.seed values, < 2^32).
 * P: the engine parameters (g_ff2 / beta replaced per iteration by the
 * schedules; V_prior_const must be set; use_prior selects the prior term of
 * V, while the moves always use alpha, fmin, fmax as the reference does).
 */
int rhmc_rj_run(rhmc_ctx* ctx, const rhmc_params* P, const rhmc_rj_config* cfg, double* q,
                int32_t* K, const uint32_t* seeds, int64_t n, const rhmc_rj_record* rec);
int rhmc_rj_run_physics(const rhmc_rj_physics* phys, const rhmc_params* P,
                        const rhmc_rj_config* cfg, double* q, int32_t* K, const uint32_t* seeds,
                        int64_t n, const rhmc_rj_record* rec);

/* Free the buffers, streams and events rhmc_rj_run keeps between runs (see
 * Retention above) on `device`, or on every device when device < 0.  A later
 * run allocates them again.  Not to be called from inside a physics callback. */
int rhmc_rj_release(int32_t device);

/* The NumPy legacy stream replica, for parity checks: n draws from
 * RandomState(seed) of `kind` into out.  kind 0: random_sample(); 1: randn();
 * 2: randint(0, (int64)a); 3: beta(a, b); 4: standard_gamma(a);
 * 5: standard_exponential(). */
int rhmc_np_draws(uint32_t seed, int32_t kind, double a, double b, int64_t n, double* out);

/* The chains' starting rows for rhmc_rj_run: rows [sum K][3] (chain after
 * chain, K[c] rows each) -> q [n][3 N_max] zero-padded.  flux_to_count > 0:
 * the rows are (mag, x, y) and the flux becomes mag2flux(mag) * flux_to_count
 * (format_q, sampler_RHMC.py:209-217, with the libm pow the reference's
 * NumPy scalars use: bit-identical); 0: the rows are already counts. */
int rhmc_rj_pack_starts(const double* rows, const int32_t* K, int64_t n, int32_t N_max,
                        double flux_to_count, double* q);

/* The same into a q whose rows are zero past 3 K_prev[c] (the previous
 * run's final rows and counts, e.g.): each row's zeros are written only up to
 * max(3 K[c], 3 K_prev[c]).  K_prev NULL, or an entry outside [1, N_max]:
 * whole rows. */
int rhmc_rj_pack_starts_padded(const double* rows, const int32_t* K, int64_t n, int32_t N_max,
                               double flux_to_count, double* q, const int32_t* K_prev);

/* The split / merge moves' Beta(beta_a, beta_b) density as the driver
 * evaluates it (scipy.stats.beta.logpdf / pdf at sampler_RHMC.py:1342, :1363,
 * :1438), for parity checks: n points x -> pdf[n], logpdf[n] (each nullable).
 * Integer exponents a - 1, b - 1 <= 8 (the reference's defaults 2, 2 and
 * RHMC-big-sim4.py's 4, 4) take the product form. */
int rhmc_rj_beta_eval(double a, double b, const double* x, int64_t n, double* pdf,
                      double* logpdf);

const char* rhmc_rj_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* RHMC_RJ_H */
