// Runtime switches of the native code: the one place that reads them.
//
// env_knob: production fallback switches, read in every build.  Each one
// restores a measured-and-kept default's predecessor and is exercised by a
// test or named in README (SA_LSTM_GANG, SA_WINO_GEO, SA_F32_WINO,
// SA_F32_WINO_POOL, SA_F32_FUSED_BWD, SA_F32_DGRAD_STACK,
// SA_F32_DGRAD_PHASE, SA_F32_POOL_SCATTER, SA_F32_POOL_BWD_BLK,
// SA_FRAMES_TILE, SA_GEMM_BL).
//
// measure_knob: the sweep / ablation knobs of experiments that were measured
// and rejected or tuned (profiles/experiments.md).  They are read only in
// builds with -DSA_MEASURE_KNOBS=1 (csrc/build.py --define SA_MEASURE_KNOBS=1
// --out PATH, loaded with SA_EXT_PATH); a production
// build always takes the default, so a stray variable on a box cannot change
// which kernels the headline runs.  bench.py reports every SA_* variable it
// was started with (config.knobs).
#pragma once

#include <cstdlib>

#ifndef SA_MEASURE_KNOBS
#define SA_MEASURE_KNOBS 0
#endif

namespace sa {

inline int env_knob(const char* name, int def) {
  const char* e = std::getenv(name);
  return (e && *e) ? std::atoi(e) : def;
}

inline int measure_knob(const char* name, int def) {
#if SA_MEASURE_KNOBS
  return env_knob(name, def);
#else
  (void)name;
  return def;
#endif
}

}  // namespace sa
