// comb_kernel / comb_latency_kernel instantiated for key plan PLA_HUGE (13 positions):
// one translation unit per plan so that the verify kernels compile in parallel.
#include "verify_kernels.h"

hipError_t launch_comb_huge(const comb_launch_args& a) { return launch_comb_plan<PLA_HUGE>(a); }

#if PBFT_COMB_STAMPS
// diagnostic build only: the per-wave phase stamps of the last comb_kernel launch of this plan (verify_kernels.h)
extern "C" int pbft_debug_comb_stamps(uint64_t* out, uint32_t waves) {
  if (waves > COMB_STAMP_WAVES) waves = COMB_STAMP_WAVES;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_comb_stamp), sizeof(uint64_t) * 8 * waves, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
