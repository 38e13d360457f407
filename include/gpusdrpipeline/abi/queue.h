/*
 * gpusdrpipeline command queues (MI355X build).
 *
 * Vtable-compatible with the reference's commandqueue/ICommandQueue.h, ICudaCommandQueue.h:23-29,
 * ICommandQueueFactory.h:49-62 and ICudaCommandQueueFactory.h:11-16 (note: the latter derives
 * from IRef non-virtually, as in the reference). A queue is one (HIP device, HIP stream); the
 * accessor names cudaDevice()/cudaStream() are kept because they are the reference's source API.
 * Streams are created non-blocking (hipStreamNonBlocking) so the queue never serialises against
 * the legacy null stream; steady-state chains on one queue can be captured into a hipGraph.
 */
#ifndef GPUSDRPIPELINE_ABI_QUEUE_H
#define GPUSDRPIPELINE_ABI_QUEUE_H

#include <gpusdrpipeline/abi/core.h>
#include <hip/hip_runtime_api.h>

class ICommandQueue : public virtual IRef {
 public:
  ABSTRACT_IREF(ICommandQueue);
};

class ICudaCommandQueue : public ICommandQueue {
 public:
  virtual int32_t cudaDevice() const noexcept = 0;
  virtual hipStream_t cudaStream() const noexcept = 0;

  ABSTRACT_IREF(ICudaCommandQueue);
};

/* Named queues, configured by JSON {"queueType": "cuda" | "hip", "cudaDevice": N}. */
class ICommandQueueFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Status create(const char* queueId, const char* parameterJson) noexcept = 0;
  [[nodiscard]] virtual bool exists(const char* queueId) noexcept = 0;
  [[nodiscard]] virtual Result<ICudaCommandQueue> getCudaCommandQueue(const char* queueId) noexcept = 0;

  ABSTRACT_IREF(ICommandQueueFactory);
};

class ICudaCommandQueueFactory : public IRef {
 public:
  virtual Result<ICudaCommandQueue> create(int32_t cudaDevice) noexcept = 0;

  ABSTRACT_IREF(ICudaCommandQueueFactory);
};

/* Current HIP device of the calling thread (reference util/CudaUtil.h:25). */
GS_EXPORT [[nodiscard]] Result<int32_t> gsGetCurrentCudaDevice() noexcept;

#endif  // GPUSDRPIPELINE_ABI_QUEUE_H
