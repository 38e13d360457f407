// HIP command queues (reference src/commandqueue: CudaCommandQueue.cpp:23-28,
// CudaCommandQueueFactory.h:14-20, CommandQueueFactory.cpp:29-94).
#pragma once

#include <gpusdrpipeline/abi/errors.h>
#include <gpusdrpipeline/abi/queue.h>

namespace gsdr_rt {

// One (device, stream). The stream is created non-blocking and destroyed with the queue.
class HipCommandQueue final : public ICudaCommandQueue {
 public:
  static Result<ICudaCommandQueue> create(int32_t device) noexcept;
  int32_t cudaDevice() const noexcept final { return mDevice; }
  hipStream_t cudaStream() const noexcept final { return mStream; }

 private:
  HipCommandQueue(int32_t device, hipStream_t stream) noexcept : mDevice(device), mStream(stream) {}
  ~HipCommandQueue() final;
  const int32_t mDevice;
  const hipStream_t mStream;
  REF_COUNTED_NO_DESTRUCTOR(HipCommandQueue);
};

class HipCommandQueueFactory final : public ICudaCommandQueueFactory {
 public:
  Result<ICudaCommandQueue> create(int32_t device) noexcept final { return HipCommandQueue::create(device); }
  REF_COUNTED(HipCommandQueueFactory);
};

// Named queues: JSON {"queueType": "cuda"|"hip", "cudaDevice": N (default 0)}.
class CommandQueueFactory final : public ICommandQueueFactory {
 public:
  explicit CommandQueueFactory(ICudaCommandQueueFactory* hipQueues) noexcept : mHipQueues(hipQueues) {}
  Status create(const char* queueId, const char* parameterJson) noexcept final;
  bool exists(const char* queueId) noexcept final;
  Result<ICudaCommandQueue> getCudaCommandQueue(const char* queueId) noexcept final;

 private:
  ICudaCommandQueueFactory* const mHipQueues;  // owned by the singleton
  REF_COUNTED(CommandQueueFactory);
};

}  // namespace gsdr_rt
