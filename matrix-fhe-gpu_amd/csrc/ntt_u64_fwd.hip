// ntt_u64_fwd.hip -- instantiates the U64 forward NTT launch plans (ntt_plans.hpp).
#include "ntt_plans.hpp"

namespace mfhe {
template int run_kind<ArithU64, TwSrcU, false>(const NttJob<TwSrcU>&, Kind, hipStream_t);
}  // namespace mfhe
