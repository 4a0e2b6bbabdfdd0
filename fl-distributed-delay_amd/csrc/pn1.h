// PerformantNet1 engine types shared by the kernels and the C-ABI.
#pragma once
#include <stdint.h>

#include "flsim.h"   // WorkerRec and the exported declarations

namespace flsim {

constexpr int SAMPLES_PER_WORKER = 128;   // main.py:43-44 --batch_size default

}  // namespace flsim
