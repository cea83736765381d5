// Forwarding header: reference include/core/trace.cuh.  The declarations live in matrix_fhe_api.hpp and are
// implemented by libmfhe.so (matrix-fhe-gpu_amd/csrc/core_api.cpp -> mfhe_trace_*, csrc/trace.hip).
#pragma once
#include "matrix_fhe_api.hpp"
