// Measurement builds.  The A/B, probe and block-stamp switches of the kernels (phases switched
// off, zeros stored instead of values, wall-clock stamps copied to the host) exist only in a
// library compiled with -DGW_MEASURE (MARLNAV_MEASURE=1 python -c 'from marlnav import _lib;
// _lib.build()'); in the release library GW_MEASURE_ENV is a null constant, so the switches are
// never read and no environment variable can make the product path skip work
// (tests/test_lib_cpu.py checks that the release .so does not even name them).
#pragma once
#include <cstdlib>

#ifdef GW_MEASURE
#define GW_MEASURE_ON 1
#define GW_MEASURE_ENV(name) std::getenv(name)
#else
#define GW_MEASURE_ON 0
#define GW_MEASURE_ENV(name) ((const char *)nullptr)
#endif

// a measurement switch bit of a kernel parameter.  The release host code never sets one (its
// GW_MEASURE_ENV reads are null), so the test is always false there; it stays a runtime test on
// purpose: folding it to a compile-time false changed the fused actors' register allocation (the
// window CNN's act kernel went from 20 B to 1.5 KB of scratch per lane and 45 -> 290 us at c4patch)
#define GW_AB(mask, bits) ((mask) & (bits))
