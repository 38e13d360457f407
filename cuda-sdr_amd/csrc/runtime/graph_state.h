// Graph stepping (SteppingDriver::doFilterGraphed): what a node tells the driver so that one
// doFilter() step of a chain can be replayed from a captured hipGraph.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace gsdr_rt {

class IGraphStepState {
 public:
  virtual ~IGraphStepState() = default;
  // The one stream every device operation of the node is enqueued on.
  virtual hipStream_t graphStream() const noexcept = 0;
  // Folds the host state that determines the node's device operations in a step (window
  // placement, constant arguments) into h. false: the node's device work cannot be replayed from a
  // capture (its launch arguments change every step, e.g. a tone's phase).
  virtual bool graphState(uint64_t& h) const noexcept = 0;
};

}  // namespace gsdr_rt
