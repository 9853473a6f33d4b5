// Skinny GEMM instantiations for EPI_F32 (see skinny_gemm_impl.h).
#include "skinny_gemm_impl.h"

int skinny_unit_f32(SKINNY_UNIT_ARGS) {
  const EpiArgs& ea = *static_cast<const EpiArgs*>(ea_p);
  if (norm)
    return launch_e<EPI_F32, true>(mt, waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  if (!norm)
    return launch_e<EPI_F32, false>(mt, waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  return (int)hipErrorInvalidValue;
}
