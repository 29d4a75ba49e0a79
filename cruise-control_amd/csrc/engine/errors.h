// Exceptions of the engine, mapped to ccmi_status at the C ABI (ccmi_api.cpp guarded()):
//   OptimizationFailure  OptimizationFailureException  -> CCMI_E_OPT_FAILURE
//   StateError           IllegalStateException         -> CCMI_E_STATE
//   Unsupported          outside the implemented scope -> CCMI_E_UNSUPPORTED
#pragma once
#include <stdexcept>

namespace ccmi {

struct OptimizationFailure : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct StateError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};

}  // namespace ccmi
