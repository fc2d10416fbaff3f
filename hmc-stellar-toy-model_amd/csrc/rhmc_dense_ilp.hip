// rhmc_dense_ilp.hip — the dense kernel's one-slot leapfrog,
// leapfrog_win_kernel<DenseG<32|48>, 1> (K <= 64 stars on 32/48-px images: B4
// and the reference's RHMC-big-sim4.py run; rhmc_dense.hpp), in a translation
// unit of its own so that it can be compiled with the max-ILP machine
// scheduler (Makefile: -mllvm -amdgpu-sched-strategy=max-ilp).  Measured on
// the whole library (profiles/r06_sched/): B4 7.74 -> 7.36 ms per launch, but
// B3's two-slot dense kernel 14.9 -> 22.4 ms and the other families 1-2 %
// slower, so only these two instantiations take it.  Scheduling does not
// change the arithmetic: results are bit-identical to the default build.
#define RHMC_KERNELS_ONLY
#include "rhmc_kernels.hip"

namespace rhmc {
template __global__ void leapfrog_win_kernel<DenseG<32>, 1>(LeapArgs);
template __global__ void leapfrog_win_kernel<DenseG<48>, 1>(LeapArgs);
}  // namespace rhmc
