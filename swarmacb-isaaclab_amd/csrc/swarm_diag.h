// swarm_diag.h — diagnostic-only build switches of the step kernel.
//
// Neither switch is set in a product build (both default to 0); the tools that
// use them build separate libraries under build/ and never ship them.
//
//   SWARM_ABLATE=mask     timing-only ablation (tools/ablate.sh): 1 skips the
//                         range-and-bearing partial, 2 the proximity partial,
//                         4 the robot pushes, 8 the arena walls, 16 the whole
//                         contact solver. Results are WRONG by design.
//   SWARM_WAVE_TIMING=1   every wave of the production step kernel records its
//                         start / end shader clock, hardware slot, work counters
//                         and per-phase clocks (tools/wave_timing.py).
#pragma once

#ifndef SWARM_ABLATE
#define SWARM_ABLATE 0
#endif

#ifndef SWARM_WAVE_TIMING
#define SWARM_WAVE_TIMING 0
#endif
