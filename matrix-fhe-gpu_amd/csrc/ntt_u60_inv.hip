// ntt_u60_inv.hip -- instantiates the U64 inverse NTT launch plans with the lazy U60 schedule (ntt_arith.hpp
// ArithU60::gs_b: X unreduced, per-register bound exponents; contexts whose moduli are all < 2^60).
#include "ntt_plans.hpp"

namespace mfhe {
template int run_kind<ArithU60, TwSrcU, true>(const NttJob<TwSrcU>&, Kind, hipStream_t);
}  // namespace mfhe
