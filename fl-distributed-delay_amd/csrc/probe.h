// Live kernel timing for bench.py: HIP events recorded on the launch stream right before and
// after selected launches (the worker-batched GEMMs and the fused aggregation), tagged with the
// launch's kernel id and its algorithmic work (FLOPs for the GEMMs, HBM bytes for aggregation).
#pragma once
#include <hip/hip_ext.h>

#include "common.h"

namespace flsim {

enum KernelId {
    K_FWD1 = 0, K_FWD2, K_FWD3, K_FWD4, K_FWD5, K_FWD6, K_L1F, K_L2F,
    K_DG2, K_DG3, K_DG4, K_DG5, K_DG6,
    K_WG1, K_WG2, K_WG3, K_WG4, K_WG5, K_WG6,
    K_L1W, K_L1D, K_L2W, K_L2D, K_AGG,
    // VGG-11 (vgg_net.hip)
    K_VF1, K_VF2, K_VF3, K_VF4, K_VF5, K_VF6, K_VF7, K_VF8, K_VL1F, K_VL2F,
    K_VDG2, K_VDG3, K_VDG4, K_VDG5, K_VDG6, K_VDG7, K_VDG8,
    K_VWG1, K_VWG2, K_VWG3, K_VWG4, K_VWG5, K_VWG6, K_VWG7, K_VWG8,
    K_VL1W, K_VL1D, K_VL2W, K_VL2D,
    // server step (server.hip): general-order aggregation, fused slab step (reference / general
    // order), slab reduction only
    K_AGG_SEQ, K_STEP, K_STEP_SEQ, K_SLABSUM, K_COUNT
};

// Event pair for the launch that follows (nullptr events when the probe is off or full).  The
// launch passes them to hipExtLaunchKernelGGL, which stamps them in the kernel's own dispatch
// packet: the measured interval is the kernel, without separate marker packets.
struct ProbeSlot {
    int slot;
    hipEvent_t start, stop;
};
ProbeSlot probe_begin();
// registers the launch (kernel id, algorithmic work); returns a C-ABI status
int probe_end(const ProbeSlot& ps, int kid, double work);

}  // namespace flsim
