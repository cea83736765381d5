// Forwarding header: reference include/core/ntt_core.cuh.  The declarations live in matrix_fhe_api.hpp and are
// implemented by libmfhe.so (matrix-fhe-gpu_amd/csrc/core_api.cpp).
#pragma once
#include "matrix_fhe_api.hpp"
