// qf_dev_hooks.h — development builds only (force-included by
// qppfuse._build.build_variant(..., dev=True); never part of libqppfuse.so).
//
// QF_STOP(phase, acc, action...): with -DQF_STOP_AT=<phase>, the kernel computes
// acc() (keeping the phase's registers live) and runs `action` (an early return
// that writes something harmless) right after that phase, so that rocprofv3's time
// and SQ_INSTS_VALU of successive stop builds give each phase's cost.  Results of
// a stop build are wrong by construction; tools/ab_run.sh only times them.
// QF_STAMPS: per-workgroup phase cycle counts into g_stamps (tools/stamps.py).
#pragma once
#ifndef QF_STOP_AT
#define QF_STOP_AT 0
#endif
#define QF_STOP(phase, acc, ...)             \
  do {                                       \
    if (QF_STOP_AT == (phase)) {             \
      const uint32_t _qf_acc = (acc)();      \
      __VA_ARGS__                            \
    }                                        \
  } while (0)

// QF_CF_SCATTER: bsort_fast_kernel's scatter stores item u at position u (consecutive
// lanes, consecutive LDS addresses: no bank conflicts) instead of its bucket position —
// the same instruction stream, wrong results; timed at stop point 24 against the
// library's scatter (round 4's conflict probe, re-run in round 6 on the 1,024-thread,
// 2^13-bucket configuration).
#ifdef QF_CF_SCATTER
#define QF_DEV_SCATTER_POS(pos, lin) (lin)
#endif
