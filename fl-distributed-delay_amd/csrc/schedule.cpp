// Epoch/worker schedule: the integer scan of main.py:119-181 (slow worker, stale FIFO,
// throttle window), generalised to any set of slow workers (delay[i] != 0).  With delays =
// [0, ..., 0, --delay] it is the reference's schedule exactly (tests pin it bit-exact against
// traces of the reference's own loop, tests/golden/schedule.npz).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "flsim.h"

#include <deque>
#include <vector>

namespace flsim {
void set_error(const char* fmt, ...);
}

struct flsim_sched {
    int32_t n;
    int32_t throttle;
    int32_t max_throttle;
    int64_t t;
    int64_t throttle_window;   // main.py:121
    int32_t slow_guy_gone;     // main.py:123
    std::vector<int32_t> delay;
    std::vector<std::deque<int64_t>> fifo;   // pesky_worker_grads per slow worker (main.py:119)
};

extern "C" {

flsim_sched* flsim_sched_create(int32_t n, const int32_t* delays, int32_t throttle,
                                int32_t max_throttle) {
    if (n <= 0 || !delays) {
        flsim::set_error("flsim_sched_create: n must be > 0 and delays non-null");
        return nullptr;
    }
    flsim_sched* s = new flsim_sched();
    s->n = n;
    s->throttle = throttle ? 1 : 0;
    s->max_throttle = max_throttle;
    s->t = 0;
    s->throttle_window = 0;
    s->slow_guy_gone = 0;
    s->delay.assign(delays, delays + n);
    s->fifo.resize(n);
    return s;
}

void flsim_sched_destroy(flsim_sched* s) { delete s; }

// Runs one epoch of the scan.
//   computes[n]      1 if worker i runs fwd_bkwd this epoch (its gradient joins S_t)
//   fast[n]          1 if worker i is a fast worker that computed (its entry is S_t and its loss
//                    is logged, main.py:171-172)
//   stale_worker / stale_src [n]: the popped FIFO entries in append order (worker, source epoch)
//   info[4] = {c_t, s_t, pushed (any slow worker stored S_t this epoch), epoch t}
// Returns 0, or 1 when the reference would raise: a slow worker with delay 0
// (FLSIM_DELAY_ZERO) at t >= 1 (ZeroDivisionError, main.py:158), or an empty weight_ups
// (IndexError in rule(), main.py:25).
int flsim_sched_epoch(flsim_sched* s, uint8_t* computes, uint8_t* fast, int32_t* stale_worker,
                      int64_t* stale_src, int64_t* info) {
    if (!s) {
        flsim::set_error("null schedule");
        return 1;
    }
    const int64_t t = s->t;
    int32_t c = 0, ns = 0, pushed = 0;
    for (int32_t i = 0; i < s->n; ++i) {
        computes[i] = 0;
        fast[i] = 0;
        const int32_t di = s->delay[i];
        if (di != 0) {                                    // main.py:150 (slow worker)
            s->slow_guy_gone = 0;                         // main.py:151
            if (di == FLSIM_DELAY_ZERO && t > 0) {        // main.py:158: t % 0
                flsim::set_error("epoch %ld: ZeroDivisionError: integer division or modulo by "
                                 "zero (--delay 0, main.py:158)", (long)t);
                return 1;
            }
            const int64_t d = di == FLSIM_DELAY_ZERO ? 0 : (di < 0 ? -(int64_t)di : (int64_t)di);
            bool popped = false;
            int64_t src = -1;
            if (t == 0) {                                 // main.py:153-157
                computes[i] = 1;
                s->fifo[i].push_back(t);
                pushed = 1;
            } else if (t % d == 0) {                      // main.py:158-162
                computes[i] = 1;
                s->fifo[i].push_back(t);
                pushed = 1;
                src = s->fifo[i].front();
                s->fifo[i].pop_front();
                popped = true;
            }
            if (popped) {                                 // main.py:164-166
                stale_worker[ns] = i;
                stale_src[ns] = src;
                ns++;
                s->slow_guy_gone = 1;
            }
        } else if (s->throttle_window <= 0) {             // main.py:168-172
            computes[i] = 1;
            fast[i] = 1;
            c++;
            if (s->throttle) {                            // main.py:174-178
                s->throttle_window = 1;
                if (!s->slow_guy_gone) {
                    s->throttle_window *= 2;
                    if (s->throttle_window > s->max_throttle) s->throttle_window = s->max_throttle;
                }
            }
        }
        if (s->throttle_window > 0) s->throttle_window -= 1;   // main.py:180-181
    }
    info[0] = c;
    info[1] = ns;
    info[2] = pushed;
    info[3] = t;
    s->t = t + 1;
    if (c + ns == 0) {
        flsim::set_error("epoch %ld: empty weight_ups (reference raises IndexError in rule())",
                         (long)t);
        return 1;
    }
    return 0;
}

// state snapshot for checkpoint/resume: {t, throttle_window, slow_guy_gone}
void flsim_sched_state(const flsim_sched* s, int64_t* out3) {
    out3[0] = s->t;
    out3[1] = s->throttle_window;
    out3[2] = s->slow_guy_gone;
}

}  // extern "C"
