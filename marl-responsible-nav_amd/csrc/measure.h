// Measurement builds.  The A/B, probe and block-stamp switches of the kernels (phases switched
// off, zeros stored instead of values, wall-clock stamps copied to the host) exist only in a
// library compiled with -DGW_MEASURE (MARLNAV_MEASURE=1 python -c 'from marlnav import _lib;
// _lib.build()'); in the release library GW_MEASURE_ENV is a null constant and GW_AB false, so
// the switches and their branches compile out and no environment variable can make the product
// path skip work (tests/test_lib_cpu.py checks that the release .so does not even name them).
#pragma once
#include <cstdlib>

#ifdef GW_MEASURE
#define GW_MEASURE_ON 1
#define GW_MEASURE_ENV(name) std::getenv(name)
#else
#define GW_MEASURE_ON 0
#define GW_MEASURE_ENV(name) ((const char *)nullptr)
#endif

// a measurement switch bit of a kernel parameter (always false in the release library)
#define GW_AB(mask, bits) (GW_MEASURE_ON && ((mask) & (bits)))
