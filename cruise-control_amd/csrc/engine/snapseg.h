// A run of scan rows taken from one broker's snapshot: (*v)[skip, end), the replicas on broker cb in the snapshot's
// order (Device::scanSegs uploads each snapshot once into the device's snapshot pool).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace ccmi {
struct SnapSeg {
  std::shared_ptr<const std::vector<int32_t>> v;
  int cb;
  size_t skip;
};
}  // namespace ccmi
