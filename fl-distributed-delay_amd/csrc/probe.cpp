// Kernel timing probe (probe.h) and its C-ABI (include/flsim.h).
#include "probe.h"

#include "flsim.h"

namespace flsim {

static const char* KNAME[K_COUNT] = {
    "conv1_fwd", "conv2_fwd", "conv3_fwd", "conv4_fwd", "conv5_fwd", "conv6_fwd", "linear1_fwd",
    "linear2_fwd", "conv2_dgrad", "conv3_dgrad", "conv4_dgrad", "conv5_dgrad", "conv6_dgrad",
    "conv1_wgrad", "conv2_wgrad", "conv3_wgrad", "conv4_wgrad", "conv5_wgrad", "conv6_wgrad",
    "linear1_wgrad", "linear1_dgrad", "linear2_wgrad", "linear2_dgrad", "aggregate_adam",
    "vgg_conv1_fwd", "vgg_conv2_fwd", "vgg_conv3_fwd", "vgg_conv4_fwd", "vgg_conv5_fwd",
    "vgg_conv6_fwd", "vgg_conv7_fwd", "vgg_conv8_fwd", "vgg_linear1_fwd", "vgg_linear2_fwd",
    "vgg_conv2_dgrad", "vgg_conv3_dgrad", "vgg_conv4_dgrad", "vgg_conv5_dgrad", "vgg_conv6_dgrad",
    "vgg_conv7_dgrad", "vgg_conv8_dgrad", "vgg_conv1_wgrad", "vgg_conv2_wgrad", "vgg_conv3_wgrad",
    "vgg_conv4_wgrad", "vgg_conv5_wgrad", "vgg_conv6_wgrad", "vgg_conv7_wgrad", "vgg_conv8_wgrad",
    "vgg_linear1_wgrad", "vgg_linear1_dgrad", "vgg_linear2_wgrad", "vgg_linear2_dgrad",
    "aggregate_adam_seq", "slab_step", "slab_step_seq", "slab_sum"};

struct Probe {
    bool on = false;
    int cap = 0, used = 0;
    hipEvent_t* ev = nullptr;
    int* kid = nullptr;
    double* work = nullptr;
};
static Probe g_probe;

ProbeSlot probe_begin() {
    if (!g_probe.on || g_probe.used >= g_probe.cap) return ProbeSlot{-1, nullptr, nullptr};
    const int u = g_probe.used;
    return ProbeSlot{u, g_probe.ev[2 * u], g_probe.ev[2 * u + 1]};
}

int probe_end(const ProbeSlot& ps, int kid, double work) {
    if (ps.slot < 0) return 0;
    g_probe.kid[ps.slot] = kid;
    g_probe.work[ps.slot] = work;
    g_probe.used = ps.slot + 1;
    return 0;
}

}  // namespace flsim

using namespace flsim;

extern "C" {

int flsim_probe_enable(int capacity) {
    if (g_probe.on) return 0;
    FLSIM_REQUIRE(capacity > 0, "capacity must be > 0");
    g_probe.ev = new hipEvent_t[2 * capacity];
    for (int i = 0; i < 2 * capacity; ++i) FLSIM_CHECK_HIP(hipEventCreate(&g_probe.ev[i]));
    g_probe.kid = new int[capacity];
    g_probe.work = new double[capacity];
    g_probe.cap = capacity;
    g_probe.used = 0;
    g_probe.on = true;
    return 0;
}

int flsim_probe_read(int* launches, double* total_ms, double* total_work) {
    for (int k = 0; k < K_COUNT; ++k) { launches[k] = 0; total_ms[k] = 0; total_work[k] = 0; }
    if (!g_probe.on) return 0;
    for (int u = 0; u < g_probe.used; ++u) {
        FLSIM_CHECK_HIP(hipEventSynchronize(g_probe.ev[2 * u + 1]));
        float ms = 0.f;
        FLSIM_CHECK_HIP(hipEventElapsedTime(&ms, g_probe.ev[2 * u], g_probe.ev[2 * u + 1]));
        launches[g_probe.kid[u]] += 1;
        total_ms[g_probe.kid[u]] += ms;
        total_work[g_probe.kid[u]] += g_probe.work[u];
    }
    g_probe.used = 0;
    return 0;
}

int flsim_probe_disable(void) {
    if (!g_probe.on) return 0;
    for (int i = 0; i < 2 * g_probe.cap; ++i) (void)hipEventDestroy(g_probe.ev[i]);
    delete[] g_probe.ev;
    delete[] g_probe.kid;
    delete[] g_probe.work;
    g_probe = Probe();
    return 0;
}

int flsim_probe_kernel_count(void) { return K_COUNT; }
const char* flsim_probe_kernel_name(int kid) { return (kid >= 0 && kid < K_COUNT) ? KNAME[kid] : ""; }

}  // extern "C"
