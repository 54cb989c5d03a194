// comb_kernel / comb_latency_kernel instantiated for key plan PLA_SMALL (32 positions):
// one translation unit per plan so that the verify kernels compile in parallel.
#include "verify_kernels.h"

hipError_t launch_comb_small(const comb_launch_args& a) { return launch_comb_plan<PLA_SMALL>(a); }
