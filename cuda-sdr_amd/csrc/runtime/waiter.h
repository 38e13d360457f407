// Keep a stream full while the host consumes results one step behind (reference
// src/filters/Waiter.cpp:34-50): recordNextAndWaitPrevious() records an event after the work
// enqueued so far and waits for the event recorded by the PREVIOUS call, so the work of the last
// call stays in flight while everything before it is complete.
#pragma once

#include <gpusdrpipeline/abi/errors.h>

#include <hip/hip_runtime.h>

#include <utility>

namespace gsdr_rt {

class Waiter {
 public:
  Waiter(int32_t device, hipStream_t stream) noexcept : mDevice(device), mStream(stream) {}
  ~Waiter() {
    if (mPrev != nullptr) (void)hipEventDestroy(mPrev);
    if (mNext != nullptr) (void)hipEventDestroy(mNext);
  }
  Waiter(const Waiter&) = delete;
  Waiter& operator=(const Waiter&) = delete;

  [[nodiscard]] Status recordNextAndWaitPrevious() noexcept {
    HipDevicePushPop push(mDevice);
    SAFE_HIP_OR_RET_STATUS(push.status());
    if (mNext == nullptr) SAFE_HIP_OR_RET_STATUS(hipEventCreateWithFlags(&mNext, hipEventDisableTiming));
    SAFE_HIP_OR_RET_STATUS(hipEventRecord(mNext, mStream));
    if (mPrev != nullptr) SAFE_HIP_OR_RET_STATUS(hipEventSynchronize(mPrev));
    std::swap(mPrev, mNext);
    return Status_Success;
  }

  // Everything enqueued so far is complete (the last call's work included).
  [[nodiscard]] Status waitAll() noexcept {
    HipDevicePushPop push(mDevice);
    SAFE_HIP_OR_RET_STATUS(push.status());
    SAFE_HIP_OR_RET_STATUS(hipStreamSynchronize(mStream));
    return Status_Success;
  }

 private:
  const int32_t mDevice;
  const hipStream_t mStream;
  hipEvent_t mPrev = nullptr;  // recorded by the previous call
  hipEvent_t mNext = nullptr;
};

}  // namespace gsdr_rt
