// Code-object preload registry (DW_PRELOAD in dw_common.h).
#include <vector>

#include "dw_common.h"

static std::vector<const void*>& preload_registry() {
  static std::vector<const void*> v;
  return v;
}

extern "C" void dw_register_preload(const void* kernel) { preload_registry().push_back(kernel); }

// Loads the code object of every registered kernel on the current device.
// Returns the number of TUs whose kernel resolved, or -hipError on the first
// failure.
extern "C" int dw_preload_code_objects() {
  int n = 0;
  for (const void* k : preload_registry()) {
    hipFuncAttributes a;
    const hipError_t e = hipFuncGetAttributes(&a, k);
    if (e != hipSuccess) return -(int)e;
    ++n;
  }
  return n;
}
