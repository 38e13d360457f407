// BaseSink / BaseSource / BaseFilter (reference src/filters/BaseSink.cpp:25-178,
// BaseSource.cpp:19-22, BaseFilter.cpp:21-28), with lazy compaction of the input window.
#include <gpusdrpipeline/abi/base_filters.h>
#include <gpusdrpipeline/abi/errors.h>

#include "buffers.h"

namespace {
constexpr size_t kInitialPortBytes = 8192;  // BaseSink.cpp:47-59
}

BaseSink::BaseSink(IRelocatableResizableBufferFactory* relocatableResizableBufferFactory,
                   IBufferSliceFactory* slicedBufferFactory, size_t inputPortCount, IMemSet* memSet)
    : mInputPortCount(inputPortCount),
      mSlicedBufferFactory(slicedBufferFactory),
      mMemSet(memSet),
      mRelocatableResizableBufferFactory(relocatableResizableBufferFactory) {
  if (inputPortCount == 0) gslogw("Sink has 0 input ports");
  GS_REQUIRE_OR_ABORT(slicedBufferFactory != nullptr || inputPortCount == 0,
                      "slicedBufferFactory cannot be null when there are input ports");
  GS_REQUIRE_OR_ABORT(relocatableResizableBufferFactory != nullptr || inputPortCount == 0,
                      "relocatableResizableBufferFactory cannot be null when there are input ports");
}

Status BaseSink::ensureInputPortsInit() noexcept {
  if (mInputPorts.size() == mInputPortCount) return Status_Success;
  try {
    std::vector<InputPort> ports;
    ports.reserve(mInputPortCount);
    for (size_t i = 0; i < mInputPortCount; ++i) {
      Ref<IRelocatableResizableBuffer> b;
      UNWRAP_OR_FWD_STATUS(b, mRelocatableResizableBufferFactory->createRelocatableBuffer(kInitialPortBytes));
      ports.push_back(InputPort{.inputBuffer = b.get().get(), .bufferCheckedOut = false});
    }
    mInputPorts = std::move(ports);
  }
  IF_CATCH_RETURN_STATUS;
  return Status_Success;
}

bool BaseSink::inputPortsInitialized() const noexcept { return mInputPorts.size() == mInputPortCount; }

Result<IBuffer> BaseSink::requestBuffer(size_t port, size_t numBytes) noexcept {
  FWD_IN_RESULT_IF_ERR(ensureInputPortsInit());
  GS_REQUIRE_OR_RET_RESULT_FMT(port < mInputPorts.size(), "Cannot request buffer: input port [%zu] out of range",
                               port);
  InputPort& p = mInputPorts[port];
  GS_REQUIRE_OR_RET_RESULT(!p.bufferCheckedOut, "Cannot request buffer - it is already checked out");
  IRelocatableResizableBuffer* b = p.inputBuffer.get();
  IBufferRange* r = b->range();
  if (r->remaining() < numBytes) {
    // retired bytes in front of the window are reclaimed first (one small D2D copy of the
    // retained history), and only then does the window grow - with 2x headroom so the next
    // steps append without compacting
    if (r->offset() != 0) FWD_IN_RESULT_IF_ERR(b->relocateUsedToStart());
    if (r->remaining() < numBytes) FWD_IN_RESULT_IF_ERR(b->resize(2 * (r->endOffset() + numBytes)));
  }
  p.bufferCheckedOut = true;
  Result<IBuffer> lent = mSlicedBufferFactory->sliceRemaining(b);
  if (lent.status != Status_Success) {
    p.bufferCheckedOut = false;
    return lent;
  }
  return lent;
}

Status BaseSink::commitBuffer(size_t port, size_t numBytes) noexcept {
  FWD_IF_ERR(ensureInputPortsInit());
  GS_REQUIRE_OR_RET_STATUS_FMT(port < mInputPorts.size(), "Cannot commit buffer: input port [%zu] out of range",
                               port);
  InputPort& p = mInputPorts[port];
  GS_REQUIRE_OR_RET_STATUS(p.bufferCheckedOut, "Cannot commit buffer - it was not checked out");
  GS_REQUIRE_OR_RET_STATUS(numBytes <= p.inputBuffer->range()->remaining(),
                           "Cannot commit buffer - the committed number of bytes exceeds its capacity");
  FWD_IF_ERR(p.inputBuffer->range()->increaseEndOffset(numBytes));
  p.bufferCheckedOut = false;
  return Status_Success;
}

Result<IBuffer> BaseSink::getPortInputBuffer(size_t port) noexcept {
  FWD_IN_RESULT_IF_ERR(ensureInputPortsInit());
  GS_REQUIRE_OR_RET_RESULT_FMT(port < mInputPorts.size(), "Input port [%zu] out of range", port);
  GS_REQUIRE_OR_RET_RESULT(!mInputPorts[port].bufferCheckedOut, "Cannot get input buffer - buffer is checked out");
  return makeRefResultNonNull<IBuffer>(mInputPorts[port].inputBuffer.get());
}

Result<const IBuffer> BaseSink::getPortInputBuffer(size_t port) const noexcept {
  GS_REQUIRE_OR_RET_RESULT_FMT(port < mInputPortCount, "Input port [%zu] out of range", port);
  GS_REQUIRE_OR_RET_RESULT(port < mInputPorts.size(), "Input buffers have not been created yet");
  GS_REQUIRE_OR_RET_RESULT(!mInputPorts[port].bufferCheckedOut, "Cannot get input buffer - buffer is checked out");
  return makeRefResultNonNull<const IBuffer>(mInputPorts[port].inputBuffer.get());
}

Status BaseSink::consumeInputBytesAndMoveUsedToStart(size_t port, size_t numBytes) noexcept {
  FWD_IF_ERR(ensureInputPortsInit());
  GS_REQUIRE_OR_RET_STATUS_FMT(port < mInputPorts.size(), "Input port [%zu] out of range", port);
  IRelocatableResizableBuffer* b = mInputPorts[port].inputBuffer.get();
  if (numBytes == 0) return Status_Success;
  FWD_IF_ERR(b->range()->increaseOffset(numBytes));
  if (b->range()->used() == 0) (void)b->range()->setUsedRange(0, 0);  // empty window: rewind for free
  return Status_Success;
}

void BaseSink::foldWindowState(uint64_t& h) const noexcept {
  auto mix = [&h](uint64_t v) { h = (h ^ v) * 0x100000001B3ull + 0x9E3779B97F4A7C15ull; };
  mix(mInputPorts.size());
  for (const InputPort& p : mInputPorts) {
    const IRelocatableResizableBuffer* b = p.inputBuffer.get();
    mix(reinterpret_cast<uintptr_t>(b->base()));
    const auto* rb = dynamic_cast<const gsdr_rt::RelocatableResizableBuffer*>(b);
    mix(rb != nullptr ? reinterpret_cast<uintptr_t>(rb->spareBase()) : 1);
    mix(b->range()->offset());
    mix(b->range()->endOffset());
    mix(b->range()->capacity());
    mix(p.bufferCheckedOut ? 1 : 0);
  }
}

IRelocatableResizableBuffer* BaseSink::inputWindow(size_t port) const noexcept {
  return port < mInputPorts.size() ? const_cast<IRelocatableResizableBuffer*>(mInputPorts[port].inputBuffer.get())
                                   : nullptr;
}

bool BaseSink::inputWindowCheckedOut(size_t port) const noexcept {
  return port < mInputPorts.size() && mInputPorts[port].bufferCheckedOut;
}

void BaseSink::setInputWindowCheckedOut(size_t port, bool checkedOut) noexcept {
  if (port < mInputPorts.size()) mInputPorts[port].bufferCheckedOut = checkedOut;
}

BaseSource::BaseSource(std::vector<ImmutableRef<IBufferCopier>>&& outputPortBufferCopiers) noexcept
    : mOutputPortBufferCopiers(std::move(outputPortBufferCopiers)) {}

IBufferCopier* BaseSource::getOutputCopier(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port < mOutputPortBufferCopiers.size(), nullptr, "Output port [%zu] out of range", port);
  return mOutputPortBufferCopiers[port].get();
}

BaseFilter::BaseFilter(IRelocatableResizableBufferFactory* relocatableResizableBufferFactory,
                       IBufferSliceFactory* slicedBufferFactory, size_t inputPortCount,
                       std::vector<ImmutableRef<IBufferCopier>>&& outputPortBufferCopiers, IMemSet* memSet) noexcept
    : BaseSink(relocatableResizableBufferFactory, slicedBufferFactory, inputPortCount, memSet),
      BaseSource(std::move(outputPortBufferCopiers)) {}
