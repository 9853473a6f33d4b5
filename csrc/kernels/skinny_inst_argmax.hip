// Skinny GEMM instantiations for EPI_ARGMAX (see skinny_gemm_impl.h).
#include "skinny_gemm_impl.h"

int skinny_unit_argmax(SKINNY_UNIT_ARGS) {
  const EpiArgs& ea = *static_cast<const EpiArgs*>(ea_p);
  if (norm)
    return launch_e<EPI_ARGMAX, true>(mt, waves, Wt, X, ldx, M, K, groups, up_off, out, ldo, eps, ea, st);
  return (int)hipErrorInvalidValue;
}
