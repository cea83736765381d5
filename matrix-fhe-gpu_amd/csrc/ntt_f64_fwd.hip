// ntt_f64_fwd.hip -- instantiates the F64 forward NTT launch plans (ntt_plans.hpp).
#include "ntt_plans.hpp"

namespace mfhe {
template int run_kind<ArithF64, TwSrcF, false>(const NttJob<TwSrcF>&, Kind, hipStream_t);
}  // namespace mfhe
