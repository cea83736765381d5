// ntt_f64_inv.hip -- instantiates the F64 inverse NTT launch plans (ntt_plans.hpp).
#include "ntt_plans.hpp"

namespace mfhe {
template int run_kind<ArithF64, TwSrcF, true>(const NttJob<TwSrcF>&, Kind, hipStream_t);
}  // namespace mfhe
