// Concrete memory / buffer objects behind the gpusdrpipeline buffer interfaces (MI355X build).
//
// Reference counterparts (src/buffers): CudaAllocator.cpp:27-110, CudaMemory.cpp, CudaBufferCopier.cpp,
// CudaMemSet.cpp, SysMem*.cpp, BufferRange.cpp, OwnedBuffer.cpp, BufferFactory.cpp, BufferSlice.cpp,
// RelocatableResizableBuffer.cpp:23-103, ResizableBuffer.cpp, BufferPool.cpp, BufferUtil.cpp.
#pragma once

#include <gpusdrpipeline/abi/buffers.h>
#include <gpusdrpipeline/abi/errors.h>
#include <gpusdrpipeline/abi/queue.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <vector>

namespace gsdr_rt {

// IMemory over any allocation; `release` frees it (device: hipFreeAsync on the owning stream).
class Memory final : public IMemory {
 public:
  Memory(uint8_t* data, size_t capacity, std::function<void()> release) noexcept
      : mData(data), mCapacity(capacity), mRelease(std::move(release)) {}
  uint8_t* data() noexcept final { return mData; }
  const uint8_t* data() const noexcept final { return mData; }
  size_t capacity() const noexcept final { return mCapacity; }

 private:
  uint8_t* const mData;
  const size_t mCapacity;
  std::function<void()> mRelease;
  ~Memory() final {
    if (mRelease) mRelease();
  }
  REF_COUNTED_NO_DESTRUCTOR(Memory);
};

class SysMemAllocator final : public IAllocator {
 public:
  Result<IMemory> allocate(size_t size) noexcept final;
  REF_COUNTED(SysMemAllocator);
};

class SysMemCopier final : public IBufferCopier {
 public:
  Status copy(void* dst, const void* src, size_t length) const noexcept final;
  REF_COUNTED(SysMemCopier);
};

class SysMemSet final : public IMemSet {
 public:
  Status memSet(void* data, uint8_t value, size_t byteCount) noexcept final;
  REF_COUNTED(SysMemSet);
};

// Device memory comes from the stream-ordered pool (hipMallocAsync) of the queue's stream;
// host memory is pinned (hipHostMalloc) so H2D/D2H copies run at PCIe DMA rate.
class HipAllocator final : public IAllocator {
 public:
  HipAllocator(ICudaCommandQueue* queue, size_t alignment, bool useHostMemory) noexcept
      : mQueue(queue), mAlignment(alignment == 0 ? 1 : alignment), mHost(useHostMemory) {}
  Result<IMemory> allocate(size_t size) noexcept final;

 private:
  ConstRef<ICudaCommandQueue> mQueue;
  const size_t mAlignment;
  const bool mHost;
  REF_COUNTED(HipAllocator);
};

class HipAllocatorFactory final : public ICudaAllocatorFactory {
 public:
  Result<IAllocator> createCudaAllocator(ICudaCommandQueue* queue, size_t alignment, bool host) noexcept final;
  REF_COUNTED(HipAllocatorFactory);
};

class HipCopier final : public IBufferCopier {
 public:
  HipCopier(ICudaCommandQueue* queue, hipMemcpyKind kind) noexcept : mQueue(queue), mKind(kind) {}
  Status copy(void* dst, const void* src, size_t length) const noexcept final;

 private:
  ConstRef<ICudaCommandQueue> mQueue;
  const hipMemcpyKind mKind;
  REF_COUNTED(HipCopier);
};

class HipCopierFactory final : public ICudaBufferCopierFactory {
 public:
  Result<IBufferCopier> createBufferCopier(ICudaCommandQueue* queue, hipMemcpyKind kind) noexcept final;
  REF_COUNTED(HipCopierFactory);
};

class HipMemSet final : public IMemSet {
 public:
  explicit HipMemSet(ICudaCommandQueue* queue) noexcept : mQueue(queue) {}
  Status memSet(void* data, uint8_t value, size_t byteCount) noexcept final;

 private:
  ConstRef<ICudaCommandQueue> mQueue;
  REF_COUNTED(HipMemSet);
};

class HipMemSetFactory final : public ICudaMemSetFactory {
 public:
  Result<IMemSet> create(ICudaCommandQueue* queue) noexcept final;
  REF_COUNTED(HipMemSetFactory);
};

class BufferRange final : public IBufferRangeMutableCapacity {
 public:
  size_t capacity() const noexcept final { return mCapacity; }
  size_t offset() const noexcept final { return mOffset; }
  size_t endOffset() const noexcept final { return mEnd; }
  Status setUsedRange(size_t offset, size_t endOffset) noexcept final;
  void setCapacity(size_t capacity) noexcept final;

 private:
  size_t mCapacity = 0, mOffset = 0, mEnd = 0;
  REF_COUNTED(BufferRange);
};

class BufferRangeFactory final : public IBufferRangeFactory {
 public:
  Result<IBufferRangeMutableCapacity> createBufferRange() const noexcept final;
  REF_COUNTED(BufferRangeFactory);
};

class OwnedBuffer final : public IBuffer {
 public:
  OwnedBuffer(IMemory* memory, IBufferRangeMutableCapacity* range) noexcept : mMemory(memory), mRange(range) {}
  uint8_t* base() noexcept final { return mMemory->data(); }
  const uint8_t* base() const noexcept final { return mMemory->data(); }
  IBufferRange* range() noexcept final { return mRange.get(); }
  const IBufferRange* range() const noexcept final { return mRange.get(); }

 private:
  ConstRef<IMemory> mMemory;
  ConstRef<IBufferRangeMutableCapacity> mRange;
  REF_COUNTED(OwnedBuffer);
};

class BufferFactory final : public IBufferFactory {
 public:
  BufferFactory(IAllocator* allocator, IBufferRangeFactory* ranges) noexcept : mAllocator(allocator), mRanges(ranges) {}
  Result<IBuffer> createBuffer(size_t size) noexcept final;

 private:
  ConstRef<IAllocator> mAllocator;
  ConstRef<IBufferRangeFactory> mRanges;
  REF_COUNTED(BufferFactory);
};

class BufferSlice final : public IBuffer {
 public:
  BufferSlice(IBuffer* parent, size_t start, IBufferRangeMutableCapacity* range) noexcept
      : mParent(parent), mStart(start), mRange(range) {}
  uint8_t* base() noexcept final { return mParent->base() + mStart; }
  const uint8_t* base() const noexcept final { return mParent->base() + mStart; }
  IBufferRange* range() noexcept final { return mRange.get(); }
  const IBufferRange* range() const noexcept final { return mRange.get(); }

 private:
  ConstRef<IBuffer> mParent;
  const size_t mStart;
  ConstRef<IBufferRangeMutableCapacity> mRange;
  REF_COUNTED(BufferSlice);
};

class BufferSliceFactory final : public IBufferSliceFactory {
 public:
  explicit BufferSliceFactory(IBufferRangeFactory* ranges) noexcept : mRanges(ranges) {}
  Result<IBuffer> slice(IBuffer* buffer, size_t start, size_t end) noexcept final;

 private:
  ConstRef<IBufferRangeFactory> mRanges;
  REF_COUNTED(BufferSliceFactory);
};

// Growable window with a spare allocation so relocate() never copies onto itself.
class RelocatableResizableBuffer final : public IRelocatableResizableBuffer {
 public:
  // the spare allocation relocate() copies into (graph stepping folds it into a window's state:
  // the first relocation allocates it)
  const void* spareBase() const noexcept { return mSpare != nullptr ? mSpare.get()->data() : nullptr; }
  static Result<IRelocatableResizableBuffer> create(size_t size, IAllocator* allocator, const IBufferCopier* copier,
                                                    const IBufferRangeFactory* ranges) noexcept;
  uint8_t* base() noexcept final { return mData == nullptr ? nullptr : mData->data(); }
  const uint8_t* base() const noexcept final { return mData == nullptr ? nullptr : mData->data(); }
  IBufferRange* range() noexcept final { return mRange.get(); }
  const IBufferRange* range() const noexcept final { return mRange.get(); }
  Status resize(size_t newSize) noexcept final;
  Status relocate(size_t dstOffset, size_t srcOffset, size_t length) noexcept final;

  // Graph replay (SteppingDriver::doFilterGraphed): the window's whole host state - which
  // allocation is live, which is the spare, the used range and the capacity - saved after a
  // captured step and reinstated when that step is replayed. Holding the allocations also keeps
  // the addresses the captured graph uses alive.
  struct Snapshot {
    Ref<IMemory> data, spare;
    size_t offset = 0, end = 0, capacity = 0;
  };
  void save(Snapshot& s) const noexcept {
    s.data = mData;
    s.spare = mSpare;
    s.offset = mRange->offset();
    s.end = mRange->endOffset();
    s.capacity = mRange->capacity();
  }
  Status restore(const Snapshot& s) noexcept {
    mData = s.data;
    mSpare = s.spare;
    mRange->setCapacity(s.capacity);
    return mRange->setUsedRange(s.offset, s.end);
  }

 private:
  RelocatableResizableBuffer(IAllocator* allocator, const IBufferCopier* copier, IBufferRangeMutableCapacity* range)
      : mAllocator(allocator), mCopier(copier), mRange(range) {}
  ConstRef<IAllocator> mAllocator;
  ConstRef<const IBufferCopier> mCopier;
  ConstRef<IBufferRangeMutableCapacity> mRange;
  Ref<IMemory> mData;
  Ref<IMemory> mSpare;
  REF_COUNTED(RelocatableResizableBuffer);
};

class RelocatableResizableBufferFactory final : public IRelocatableResizableBufferFactory {
 public:
  RelocatableResizableBufferFactory(IAllocator* allocator, const IBufferCopier* copier, IBufferRangeFactory* ranges)
      : mAllocator(allocator), mCopier(copier), mRanges(ranges) {}
  Result<IRelocatableResizableBuffer> createRelocatableBuffer(size_t size) const noexcept final {
    return RelocatableResizableBuffer::create(size, mAllocator, mCopier, mRanges);
  }

 private:
  ConstRef<IAllocator> mAllocator;
  ConstRef<const IBufferCopier> mCopier;
  ConstRef<IBufferRangeFactory> mRanges;
  REF_COUNTED(RelocatableResizableBufferFactory);
};

// A plain resizable buffer (grows by reallocating and copying the whole capacity).
class ResizableBuffer final : public IResizableBuffer {
 public:
  ResizableBuffer(IAllocator* allocator, const IBufferCopier* copier, IBufferRangeMutableCapacity* range)
      : mAllocator(allocator), mCopier(copier), mRange(range) {}
  uint8_t* base() noexcept final { return mData == nullptr ? nullptr : mData->data(); }
  const uint8_t* base() const noexcept final { return mData == nullptr ? nullptr : mData->data(); }
  IBufferRange* range() noexcept final { return mRange.get(); }
  const IBufferRange* range() const noexcept final { return mRange.get(); }
  Status resize(size_t newSize) noexcept final;

 private:
  ConstRef<IAllocator> mAllocator;
  ConstRef<const IBufferCopier> mCopier;
  ConstRef<IBufferRangeMutableCapacity> mRange;
  Ref<IMemory> mData;
  REF_COUNTED(ResizableBuffer);
};

class ResizableBufferFactory final : public IResizableBufferFactory {
 public:
  ResizableBufferFactory(IAllocator* allocator, const IBufferCopier* copier, IBufferRangeFactory* ranges)
      : mAllocator(allocator), mCopier(copier), mRanges(ranges) {}
  Result<IResizableBuffer> createResizableBuffer(size_t size) noexcept final;

 private:
  ConstRef<IAllocator> mAllocator;
  ConstRef<const IBufferCopier> mCopier;
  ConstRef<IBufferRangeFactory> mRanges;
  REF_COUNTED(ResizableBufferFactory);
};

// Bounded pool of equally sized buffers; getBuffer() blocks while all are lent out.
class BufferPool final : public IBufferPool {
 public:
  BufferPool(size_t maxBuffers, size_t bufferSize, IBufferFactory* factory)
      : mMax(maxBuffers), mSize(bufferSize), mFactory(factory) {}
  size_t getBufferSize() const noexcept final { return mSize; }
  Result<IBuffer> getBuffer() noexcept final { return take(true); }
  Result<IBuffer> tryGetBuffer() noexcept final { return take(false); }

 private:
  Result<IBuffer> take(bool block) noexcept;
  const size_t mMax, mSize;
  ConstRef<IBufferFactory> mFactory;
  std::mutex mLock;
  std::condition_variable mCv;
  std::vector<ImmutableRef<IBuffer>> mAll;
  std::vector<bool> mLent;
  REF_COUNTED(BufferPool);
};

class BufferPoolFactory final : public IBufferPoolFactory {
 public:
  BufferPoolFactory(size_t maxBuffers, IBufferFactory* factory) : mMax(maxBuffers), mFactory(factory) {}
  Result<IBufferPool> createBufferPool(size_t bufferSize) noexcept final {
    return makeRefResultNonNull<IBufferPool>(new (std::nothrow) BufferPool(mMax, bufferSize, mFactory));
  }

 private:
  const size_t mMax;
  ConstRef<IBufferFactory> mFactory;
  REF_COUNTED(BufferPoolFactory);
};

class BufferUtil final : public IBufferUtil {
 public:
  Status appendToBuffer(IBuffer* buffer, const void* src, size_t count,
                        const IBufferCopier* copier) const noexcept final;
  Status readFromBuffer(void* dst, IBuffer* buffer, size_t count, const IBufferCopier* copier) const noexcept final;
  Status moveFromBuffer(IBuffer* dst, IBuffer* src, size_t count, const IBufferCopier* copier) const noexcept final;
  REF_COUNTED(BufferUtil);
};

}  // namespace gsdr_rt
