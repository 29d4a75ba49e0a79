// Exceptions of the engine, mapped to ccmi_status at the C ABI (ccmi_api.cpp guarded()):
//   OptimizationFailure  OptimizationFailureException  -> CCMI_E_OPT_FAILURE
//   StateError           IllegalStateException         -> CCMI_E_STATE
//   Unsupported          outside the implemented scope -> CCMI_E_UNSUPPORTED
#pragma once
#include <stdexcept>
#include <string>

#include "ccmi.h"

namespace ccmi {

// ProvisionRecommendation.Builder(status) with every optional field unset (-1)
inline ccmi_provision_recommendation provisionRec(int status = CCMI_PROVISION_UNDER_PROVISIONED) {
  ccmi_provision_recommendation r{};
  r.status = status;
  r.num_brokers = r.num_racks = r.num_disks = r.num_partitions = r.typical_broker_id = r.resource = -1;
  r.typical_broker_capacity = r.total_capacity = -1.0;
  return r;
}
inline ccmi_provision_recommendation underBrokers(int n, int resource = -1) {
  ccmi_provision_recommendation r = provisionRec();
  r.num_brokers = n;
  r.resource = resource;
  return r;
}
inline ccmi_provision_response provisionResponse(int status) {
  ccmi_provision_response p{};
  p.status = status;
  p.recommendation = provisionRec(0);
  return p;
}
inline ccmi_provision_response provisionResponse(int status, const ccmi_provision_recommendation& r) {
  ccmi_provision_response p{};
  p.status = status;
  p.has_recommendation = 1;
  p.recommendation = r;
  return p;
}

// OptimizationFailureException with its (optional) ProvisionRecommendation
struct OptimizationFailure : std::runtime_error {
  explicit OptimizationFailure(const std::string& m) : std::runtime_error(m) {}
  OptimizationFailure(const std::string& m, const ccmi_provision_recommendation& r)
      : std::runtime_error(m), hasRec(true), rec(r) {}
  bool hasRec = false;
  ccmi_provision_recommendation rec{};
};
struct StateError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// the message ccmi_last_error returns (ccmi_api.cpp)
void setLastError(const std::string& msg);

}  // namespace ccmi
