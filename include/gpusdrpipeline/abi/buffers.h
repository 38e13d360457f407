/*
 * gpusdrpipeline buffer interfaces (MI355X build).
 *
 * Vtable-compatible with the reference's include/gpusdrpipeline/buffers/I*.h:
 *   IBufferRange (IBufferRange.h:29-84), IBufferRangeMutableCapacity, IBuffer (IBuffer.h:26-48),
 *   IBufferCopier, IAllocator, IMemSet, IBufferFactory, IBufferSliceFactory (:24-58),
 *   IBufferRangeFactory, IResizable / IRelocatable, IResizableBuffer, IRelocatableResizableBuffer,
 *   their factories, IBufferPool(+Factory), IBufferUtil and the HIP-backed factories
 *   ICudaAllocatorFactory / ICudaBufferCopierFactory / ICudaMemSetFactory.
 *
 * The HIP-backed factories keep their reference names (the names are part of the source API),
 * but take hipMemcpyKind: its enumerators have the same values (0..4) as cudaMemcpyKind.
 */
#ifndef GPUSDRPIPELINE_ABI_BUFFERS_H
#define GPUSDRPIPELINE_ABI_BUFFERS_H

#include <gpusdrpipeline/abi/core.h>
#include <hip/hip_runtime_api.h>

class ICommandQueue;
class ICudaCommandQueue;

/* [offset, endOffset) is the used region of a buffer of `capacity` bytes. */
class IBufferRange : public virtual IRef {
 public:
  [[nodiscard]] virtual size_t capacity() const noexcept = 0;
  [[nodiscard]] virtual size_t offset() const noexcept = 0;
  [[nodiscard]] virtual size_t endOffset() const noexcept = 0;
  [[nodiscard]] virtual Status setUsedRange(size_t offset, size_t endOffset) noexcept = 0;

  [[nodiscard]] virtual size_t used() const noexcept { return endOffset() - offset(); }
  [[nodiscard]] virtual size_t remaining() const noexcept { return capacity() - endOffset(); }
  [[nodiscard]] virtual bool hasRemaining() const noexcept { return remaining() > 0; }

  void clearRange() noexcept { (void)setUsedRange(0, 0); }

  [[nodiscard]] Status increaseOffset(size_t by) {
    const size_t next = offset() + by;
    if (next > endOffset()) {
      gsloge("New start offset [%zu] exceeds the end offset [%zu]", next, endOffset());
      return Status_InvalidArgument;
    }
    return setUsedRange(next, endOffset());
  }

  [[nodiscard]] Status increaseEndOffset(size_t by) {
    const size_t next = endOffset() + by;
    if (next > capacity()) {
      gsloge("New end offset [%zu] exceeds the capacity [%zu]", next, capacity());
      return Status_InvalidArgument;
    }
    return setUsedRange(offset(), next);
  }

  ABSTRACT_IREF(IBufferRange);
};

class IBufferRangeMutableCapacity : public IBufferRange {
 public:
  virtual void setCapacity(size_t capacity) noexcept = 0;

  ABSTRACT_IREF(IBufferRangeMutableCapacity);
};

class IBuffer : public virtual IRef {
 public:
  [[nodiscard]] virtual uint8_t* base() noexcept = 0;
  [[nodiscard]] virtual const uint8_t* base() const noexcept = 0;
  [[nodiscard]] virtual IBufferRange* range() noexcept = 0;
  [[nodiscard]] virtual const IBufferRange* range() const noexcept = 0;

  template <class T = uint8_t>
  [[nodiscard]] const T* readPtr() const noexcept {
    return reinterpret_cast<const T*>(base() + range()->offset());
  }
  template <class T = uint8_t>
  [[nodiscard]] T* writePtr() noexcept {
    return reinterpret_cast<T*>(base() + range()->endOffset());
  }

  ABSTRACT_IREF(IBuffer);
};

class IBufferCopier : public virtual IRef {
 public:
  [[nodiscard]] virtual Status copy(void* dst, const void* src, size_t length) const noexcept = 0;

  ABSTRACT_IREF(IBufferCopier);
};

class IAllocator : public virtual IRef {
 public:
  /* At least `size` bytes; implementations may round up (vector-width padding). */
  [[nodiscard]] virtual Result<IMemory> allocate(size_t size) noexcept = 0;

  ABSTRACT_IREF(IAllocator);
};

class IAllocatorFactory : public virtual IRef {
 public:
  virtual Result<IAllocator> create(ICommandQueue* forCommandQueue) = 0;

  ABSTRACT_IREF(IAllocatorFactory);
};

class IMemSet : public virtual IRef {
 public:
  [[nodiscard]] virtual Status memSet(void* data, uint8_t value, size_t byteCount) noexcept = 0;

  ABSTRACT_IREF(IMemSet);
};

class IBufferFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IBuffer> createBuffer(size_t size) noexcept = 0;

  ABSTRACT_IREF(IBufferFactory);
};

class IBufferSliceFactory : public virtual IRef {
 public:
  /* A view of [sliceStartOffset, sliceEndOffset) of bufferToSlice whose used range is the
   * overlap with bufferToSlice's used range (re-based to the slice). */
  [[nodiscard]] virtual Result<IBuffer> slice(IBuffer* bufferToSlice, size_t sliceStartOffset,
                                              size_t sliceEndOffset) noexcept = 0;

  /* The unused tail [endOffset, capacity) of a buffer as an empty buffer. */
  [[nodiscard]] Result<IBuffer> sliceRemaining(IBuffer* bufferToSlice) {
    return slice(bufferToSlice, bufferToSlice->range()->endOffset(), bufferToSlice->range()->capacity());
  }

  ABSTRACT_IREF(IBufferSliceFactory);
};

class IBufferRangeFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IBufferRangeMutableCapacity> createBufferRange() const noexcept = 0;

  [[nodiscard]] Result<IBufferRangeMutableCapacity> createBufferRangeWithCapacity(size_t capacity) const {
    IBufferRangeMutableCapacity* r;
    UNWRAP_OR_FWD_RESULT(r, createBufferRange());
    r->setCapacity(capacity);
    return makeRefResultNonNull(r);
  }

 protected:
  ABSTRACT_IREF(IBufferRangeFactory);
};

class IResizable : public virtual IRef {
 public:
  [[nodiscard]] virtual Status resize(size_t newSize) noexcept = 0;

  ABSTRACT_IREF(IResizable);
};

class IRelocatable : public virtual IRef {
 public:
  [[nodiscard]] virtual Status relocate(size_t dstOffset, size_t srcOffset, size_t length) noexcept = 0;

  ABSTRACT_IREF(IRelocatable);
};

class IResizableBuffer : public IBuffer, public IResizable {
 public:
  [[nodiscard]] Status ensureMinSize(size_t minSize) noexcept {
    return range()->capacity() < minSize ? resize(minSize) : Status_Success;
  }

  ABSTRACT_IREF(IResizableBuffer);
};

class IRelocatableResizableBuffer : public IRelocatable, public IResizableBuffer {
 public:
  [[nodiscard]] Status relocateUsedToStart() noexcept { return relocate(0, range()->offset(), range()->used()); }

  ABSTRACT_IREF(IRelocatableResizableBuffer);
};

class IResizableBufferFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IResizableBuffer> createResizableBuffer(size_t size) noexcept = 0;

  ABSTRACT_IREF(IResizableBufferFactory);
};

class IRelocatableResizableBufferFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IRelocatableResizableBuffer> createRelocatableBuffer(size_t size) const noexcept = 0;

  ABSTRACT_IREF(IRelocatableResizableBufferFactory);
};

class IRelocatableCudaBufferFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IRelocatableResizableBuffer> createCudaBuffer(size_t minSize,
                                                                             ICudaCommandQueue* commandQueue,
                                                                             size_t alignment,
                                                                             bool useHostMemory) noexcept = 0;

  ABSTRACT_IREF(IRelocatableCudaBufferFactory);
};

class IBufferPool : public virtual IRef {
 public:
  [[nodiscard]] virtual size_t getBufferSize() const noexcept = 0;
  [[nodiscard]] virtual Result<IBuffer> getBuffer() noexcept = 0;     // may block
  [[nodiscard]] virtual Result<IBuffer> tryGetBuffer() noexcept = 0;  // never blocks

  ABSTRACT_IREF(IBufferPool);
};

class IBufferPoolFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IBufferPool> createBufferPool(size_t bufferSize) noexcept = 0;

  ABSTRACT_IREF(IBufferPoolFactory);
};

class IBufferUtil : public virtual IRef {
 public:
  [[nodiscard]] virtual Status appendToBuffer(IBuffer* buffer, const void* src, size_t count,
                                              const IBufferCopier* bufferCopier) const noexcept = 0;
  [[nodiscard]] virtual Status readFromBuffer(void* dst, IBuffer* buffer, size_t count,
                                              const IBufferCopier* bufferCopier) const noexcept = 0;
  [[nodiscard]] virtual Status moveFromBuffer(IBuffer* dst, IBuffer* src, size_t count,
                                              const IBufferCopier* bufferCopier) const noexcept = 0;

  ABSTRACT_IREF(IBufferUtil);
};

/* Device (hipMallocAsync on the queue's stream) or pinned host (hipHostMalloc) memory,
 * base address rounded up to `alignment`. */
class ICudaAllocatorFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IAllocator> createCudaAllocator(ICudaCommandQueue* commandQueue, size_t alignment,
                                                               bool useHostMemory) noexcept = 0;

  ABSTRACT_IREF(ICudaAllocatorFactory);
};

/* hipMemcpyAsync of a fixed kind on the queue's stream. */
class ICudaBufferCopierFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IBufferCopier> createBufferCopier(ICudaCommandQueue* commandQueue,
                                                                 hipMemcpyKind memcpyKind) noexcept = 0;

  ABSTRACT_IREF(ICudaBufferCopierFactory);
};

/* hipMemsetAsync on the queue's stream. */
class ICudaMemSetFactory : public virtual IRef {
 public:
  [[nodiscard]] virtual Result<IMemSet> create(ICudaCommandQueue* commandQueue) noexcept = 0;

  ABSTRACT_IREF(ICudaMemSetFactory);
};

#endif  // GPUSDRPIPELINE_ABI_BUFFERS_H
