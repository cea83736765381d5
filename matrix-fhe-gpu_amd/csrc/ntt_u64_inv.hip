// ntt_u64_inv.hip -- instantiates the U64 inverse NTT launch plans (ntt_plans.hpp).
#include "ntt_plans.hpp"

namespace mfhe {
template int run_kind<ArithU64, TwSrcU, true>(const NttJob<TwSrcU>&, Kind, hipStream_t);
}  // namespace mfhe
