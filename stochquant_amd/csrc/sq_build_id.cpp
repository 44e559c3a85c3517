// sq_build_id.cpp -- identity of the compiled code in this libstochquant.so.
// stochquant_amd/build.py compiles this file last, defining SQ_BUILD_ID as
// "phi4:<sha256/16 of sq_phi4.hip.o> lib:<sha256/16 of every object>": the
// phi4 part changes exactly when the φ⁴ step kernels' code object does, so a
// PMC record taken from one build (profiles/*/driver_profile.json) can be
// refused by bench.py when the library that runs is a different one.
#include "../../include/stochquant.h"

#ifndef SQ_BUILD_ID
#define SQ_BUILD_ID "unknown"
#endif

extern "C" const char *sq_build_id(void) { return SQ_BUILD_ID; }
