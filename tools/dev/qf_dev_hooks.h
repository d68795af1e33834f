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
