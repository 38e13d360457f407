// Graph stepping (SteppingDriver::doFilterGraphed): what a node tells the driver so that one
// doFilter() step of a chain can be replayed from a captured hipGraph without re-running the
// step's host logic.
#pragma once

#include "buffers.h"

#include <gpusdrpipeline/abi/base_filters.h>

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

namespace gsdr_rt {

// A node's host state after a step: every input window's snapshot and checkout flag.
struct GraphNodeState {
  std::vector<RelocatableResizableBuffer::Snapshot> windows;
  std::vector<bool> checkedOut;
};

class IGraphStepState {
 public:
  virtual ~IGraphStepState() = default;
  // The one stream every device operation of the node is enqueued on.
  virtual hipStream_t graphStream() const noexcept = 0;
  // Folds the host state that determines the node's device operations in a step (window
  // placement, constant arguments) into h. false: the node's device work cannot be replayed from a
  // capture (its launch arguments change every step, e.g. a tone's phase).
  virtual bool graphState(uint64_t& h) const noexcept = 0;
  // The node's host state after a captured step / reinstating it when the step is replayed. A step
  // from a given graphState() is deterministic, so its end state is too.
  virtual bool saveStepState(GraphNodeState& out) const noexcept = 0;
  virtual Status restoreStepState(const GraphNodeState& in) noexcept = 0;
};

// The common implementation for nodes whose only host state is their input windows (BaseSink).
inline bool saveSinkWindows(const BaseSink& sink, GraphNodeState& out) noexcept {
  try {
    out.windows.assign(sink.inputWindowCount(), {});
    out.checkedOut.assign(sink.inputWindowCount(), false);
  } catch (...) {
    return false;
  }
  for (size_t p = 0; p < sink.inputWindowCount(); ++p) {
    const auto* w = dynamic_cast<const RelocatableResizableBuffer*>(sink.inputWindow(p));
    if (w == nullptr) return false;
    w->save(out.windows[p]);
    out.checkedOut[p] = sink.inputWindowCheckedOut(p);
  }
  return true;
}

inline Status restoreSinkWindows(BaseSink& sink, const GraphNodeState& in) noexcept {
  if (in.windows.size() != sink.inputWindowCount()) return Status_InvalidState;
  for (size_t p = 0; p < in.windows.size(); ++p) {
    auto* w = dynamic_cast<RelocatableResizableBuffer*>(sink.inputWindow(p));
    if (w == nullptr) return Status_InvalidState;
    FWD_IF_ERR(w->restore(in.windows[p]));
    sink.setInputWindowCheckedOut(p, in.checkedOut[p]);
  }
  return Status_Success;
}

}  // namespace gsdr_rt
