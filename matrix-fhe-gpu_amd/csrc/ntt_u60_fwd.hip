// ntt_u60_fwd.hip -- instantiates the U64 forward NTT launch plans with the lazy U60 schedule (ntt_arith.hpp
// ArithU60: contexts whose moduli are all < 2^60).
#include "ntt_plans.hpp"

namespace mfhe {
template int run_kind<ArithU60, TwSrcU, false>(const NttJob<TwSrcU>&, Kind, hipStream_t);
}  // namespace mfhe
