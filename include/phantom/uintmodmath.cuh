// Forwarding header: phantom-fhe include/uintmodmath.cuh (the subset Matrix-FHE-GPU binds).  Declarations in
// phantom_api.hpp, implemented by libmfhe.so (matrix-fhe-gpu_amd/csrc/core_api.cpp).
#pragma once
#include "phantom_api.hpp"
