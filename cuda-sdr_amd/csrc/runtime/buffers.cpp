#include "buffers.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace gsdr_rt {

// ---- system memory ------------------------------------------------------------------------------
Result<IMemory> SysMemAllocator::allocate(size_t size) noexcept {
  constexpr size_t kAlign = 64;
  const size_t rounded = (std::max<size_t>(size, 1) + kAlign - 1) / kAlign * kAlign;
  void* p = aligned_alloc(kAlign, rounded);
  if (p == nullptr) return ERR_RESULT(Status_OutOfMemory);
  return makeRefResultNonNull<IMemory>(
      new (std::nothrow) Memory(static_cast<uint8_t*>(p), size == 0 ? 0 : rounded, [p]() { free(p); }));
}

Status SysMemCopier::copy(void* dst, const void* src, size_t length) const noexcept {
  if (length != 0) memmove(dst, src, length);
  return Status_Success;
}

Status SysMemSet::memSet(void* data, uint8_t value, size_t byteCount) noexcept {
  if (byteCount != 0) memset(data, value, byteCount);
  return Status_Success;
}

// ---- HIP memory (CudaAllocator.cpp:32-110 counterpart) -----------------------------------------------
Result<IMemory> HipAllocator::allocate(size_t size) noexcept {
  if (size == 0) return makeRefResultNonNull<IMemory>(new (std::nothrow) Memory(nullptr, 0, nullptr));
  if (size > (size_t)INT64_MAX) return ERR_RESULT(Status_InvalidArgument);
  const int32_t device = mQueue->cudaDevice();
  hipStream_t stream = mQueue->cudaStream();
  HIP_DEV_PUSH_POP_OR_RET_RESULT(device);
  const size_t usable = (size + mAlignment - 1) / mAlignment * mAlignment;
  const size_t allocSize = usable + mAlignment - 1;
  void* raw = nullptr;
  if (mHost) {
    SAFE_HIP_OR_RET_RESULT(hipHostMalloc(&raw, allocSize, hipHostMallocDefault));
  } else {
    SAFE_HIP_OR_RET_RESULT(hipMallocAsync(&raw, allocSize, stream));
  }
  const uintptr_t a = (reinterpret_cast<uintptr_t>(raw) + mAlignment - 1) / mAlignment * mAlignment;
  std::function<void()> release;
  if (mHost) {
    // pinned host memory may still be the source/target of an in-flight copy on the stream
    release = [raw, device, stream]() {
      HipDevicePushPop push(device);
      (void)hipStreamSynchronize(stream);
      SAFE_HIP_WARN_ONLY(hipHostFree(raw));
    };
  } else {
    release = [raw, device, stream]() {
      HipDevicePushPop push(device);
      SAFE_HIP_WARN_ONLY(hipFreeAsync(raw, stream));
    };
  }
  gslogd("HIP %s allocation of %zu bytes (alignment %zu) on device %d", mHost ? "pinned host" : "device", size,
         mAlignment, device);
  return makeRefResultNonNull<IMemory>(new (std::nothrow)
                                           Memory(reinterpret_cast<uint8_t*>(a), usable, std::move(release)));
}

Result<IAllocator> HipAllocatorFactory::createCudaAllocator(ICudaCommandQueue* queue, size_t alignment,
                                                            bool host) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  return makeRefResultNonNull<IAllocator>(new (std::nothrow) HipAllocator(queue, alignment, host));
}

Status HipCopier::copy(void* dst, const void* src, size_t length) const noexcept {
  if (length == 0) return Status_Success;
  HIP_DEV_PUSH_POP_OR_RET_STATUS(mQueue->cudaDevice());
  SAFE_HIP_OR_RET_STATUS(hipMemcpyAsync(dst, src, length, mKind, mQueue->cudaStream()));
  return Status_Success;
}

Result<IBufferCopier> HipCopierFactory::createBufferCopier(ICudaCommandQueue* queue, hipMemcpyKind kind) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  return makeRefResultNonNull<IBufferCopier>(new (std::nothrow) HipCopier(queue, kind));
}

Status HipMemSet::memSet(void* data, uint8_t value, size_t byteCount) noexcept {
  if (byteCount == 0) return Status_Success;
  HIP_DEV_PUSH_POP_OR_RET_STATUS(mQueue->cudaDevice());
  SAFE_HIP_OR_RET_STATUS(hipMemsetAsync(data, value, byteCount, mQueue->cudaStream()));
  return Status_Success;
}

Result<IMemSet> HipMemSetFactory::create(ICudaCommandQueue* queue) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  return makeRefResultNonNull<IMemSet>(new (std::nothrow) HipMemSet(queue));
}

// ---- ranges and buffers ---------------------------------------------------------------------------
Status BufferRange::setUsedRange(size_t offset, size_t endOffset) noexcept {
  GS_REQUIRE_OR_RET_STATUS_FMT(offset <= endOffset, "offset [%zu] > end offset [%zu]", offset, endOffset);
  GS_REQUIRE_OR_RET_STATUS_FMT(endOffset <= mCapacity, "end offset [%zu] > capacity [%zu]", endOffset, mCapacity);
  mOffset = offset;
  mEnd = endOffset;
  return Status_Success;
}

void BufferRange::setCapacity(size_t capacity) noexcept {
  mCapacity = capacity;
  mEnd = std::min(mEnd, capacity);
  mOffset = std::min(mOffset, mEnd);
}

Result<IBufferRangeMutableCapacity> BufferRangeFactory::createBufferRange() const noexcept {
  return makeRefResultNonNull<IBufferRangeMutableCapacity>(new (std::nothrow) BufferRange());
}

Result<IBuffer> BufferFactory::createBuffer(size_t size) noexcept {
  Ref<IMemory> memory;
  Ref<IBufferRangeMutableCapacity> range;
  UNWRAP_OR_FWD_RESULT(memory, mAllocator->allocate(size));
  UNWRAP_OR_FWD_RESULT(range, mRanges->createBufferRange());
  range->setCapacity(memory->capacity());
  return makeRefResultNonNull<IBuffer>(new (std::nothrow) OwnedBuffer(memory.get(), range.get()));
}

// BufferSlice.cpp:27-186: the slice's used range is the overlap of [start, end) with the
// parent's used range, re-based to the slice (an empty overlap gives [0, 0)).
Result<IBuffer> BufferSliceFactory::slice(IBuffer* buffer, size_t start, size_t end) noexcept {
  NON_NULL_PARAM_OR_RET(buffer);
  GS_REQUIRE_OR_RET_RESULT_FMT(start <= end, "slice start [%zu] > end [%zu]", start, end);
  GS_REQUIRE_OR_RET_RESULT_FMT(end <= buffer->range()->capacity(), "slice end [%zu] > capacity [%zu]", end,
                               buffer->range()->capacity());
  Ref<IBufferRangeMutableCapacity> range;
  UNWRAP_OR_FWD_RESULT(range, mRanges->createBufferRange());
  range->setCapacity(end - start);
  const size_t lo = std::max(buffer->range()->offset(), start);
  const size_t hi = std::min(buffer->range()->endOffset(), end);
  if (lo < hi) FWD_IN_RESULT_IF_ERR(range->setUsedRange(lo - start, hi - start));
  return makeRefResultNonNull<IBuffer>(new (std::nothrow) BufferSlice(buffer, start, range.get()));
}

// ---- relocatable window (RelocatableResizableBuffer.cpp:23-103 counterpart) ---------------------------
Result<IRelocatableResizableBuffer> RelocatableResizableBuffer::create(size_t size, IAllocator* allocator,
                                                                       const IBufferCopier* copier,
                                                                       const IBufferRangeFactory* ranges) noexcept {
  NON_NULL_PARAM_OR_RET(allocator);
  NON_NULL_PARAM_OR_RET(copier);
  NON_NULL_PARAM_OR_RET(ranges);
  Ref<IBufferRangeMutableCapacity> range;
  UNWRAP_OR_FWD_RESULT(range, ranges->createBufferRange());
  auto* b = new (std::nothrow) RelocatableResizableBuffer(allocator, copier, range.get());
  NON_NULL_OR_RET(b);
  const Status st = b->resize(size);
  if (st != Status_Success) {
    b->unref();
    return ERR_RESULT(st);
  }
  return makeRefResultNonNull<IRelocatableResizableBuffer>(b);
}

// Grows the allocation, preserving the USED bytes at their offsets (the reference copies the
// whole old capacity). The spare allocation is dropped and re-created lazily by relocate().
Status RelocatableResizableBuffer::resize(size_t newSize) noexcept {
  if (newSize <= mRange->capacity() && mData != nullptr) return Status_Success;
  Ref<IMemory> fresh;
  UNWRAP_OR_FWD_STATUS(fresh, mAllocator->allocate(std::max<size_t>(newSize, 1)));
  if (mData != nullptr && mRange->used() != 0) {
    FWD_IF_ERR(mCopier->copy(fresh->data() + mRange->offset(), mData->data() + mRange->offset(), mRange->used()));
  }
  mSpare.reset();
  mData = fresh;
  mRange->setCapacity(fresh->capacity());
  return Status_Success;
}

Status RelocatableResizableBuffer::relocate(size_t dstOffset, size_t srcOffset, size_t length) noexcept {
  const size_t cap = mRange->capacity();
  GS_REQUIRE_OR_RET_STATUS_FMT(dstOffset + length <= cap, "relocate target [%zu + %zu] beyond capacity [%zu]",
                               dstOffset, length, cap);
  GS_REQUIRE_OR_RET_STATUS_FMT(srcOffset + length <= cap, "relocate source [%zu + %zu] beyond capacity [%zu]",
                               srcOffset, length, cap);
  if (length > 0 && dstOffset != srcOffset) {
    if (mSpare == nullptr || mSpare->capacity() < cap) UNWRAP_OR_FWD_STATUS(mSpare, mAllocator->allocate(cap));
    // copy into the spare allocation and swap: source and destination never overlap
    FWD_IF_ERR(mCopier->copy(mSpare->data() + dstOffset, mData->data() + srcOffset, length));
    Ref<IMemory> t = mData;
    mData = mSpare;
    mSpare = t;
  }
  // [dstOffset, dstOffset + length) (the reference sets (dstOffset, length), correct only for 0)
  return mRange->setUsedRange(dstOffset, dstOffset + length);
}

Status ResizableBuffer::resize(size_t newSize) noexcept {
  if (newSize <= mRange->capacity() && mData != nullptr) return Status_Success;
  Ref<IMemory> fresh;
  UNWRAP_OR_FWD_STATUS(fresh, mAllocator->allocate(std::max<size_t>(newSize, 1)));
  if (mData != nullptr && mRange->capacity() != 0) FWD_IF_ERR(mCopier->copy(fresh->data(), mData->data(),
                                                                           mRange->capacity()));
  mData = fresh;
  mRange->setCapacity(fresh->capacity());
  return Status_Success;
}

Result<IResizableBuffer> ResizableBufferFactory::createResizableBuffer(size_t size) noexcept {
  Ref<IBufferRangeMutableCapacity> range;
  UNWRAP_OR_FWD_RESULT(range, mRanges->createBufferRange());
  auto* b = new (std::nothrow) ResizableBuffer(mAllocator, mCopier, range.get());
  NON_NULL_OR_RET(b);
  const Status st = b->resize(size);
  if (st != Status_Success) {
    b->unref();
    return ERR_RESULT(st);
  }
  return makeRefResultNonNull<IResizableBuffer>(b);
}

// ---- pool -----------------------------------------------------------------------------------------
namespace {
// Lends a pool buffer; when the borrower drops the last reference the slot becomes free again.
class PoolLease final : public IBuffer {
 public:
  PoolLease(IBuffer* inner, std::function<void()> onRelease) : mInner(inner), mOnRelease(std::move(onRelease)) {}
  uint8_t* base() noexcept final { return mInner->base(); }
  const uint8_t* base() const noexcept final { return mInner->base(); }
  IBufferRange* range() noexcept final { return mInner->range(); }
  const IBufferRange* range() const noexcept final { return mInner->range(); }

 private:
  ConstRef<IBuffer> mInner;
  std::function<void()> mOnRelease;
  ~PoolLease() final {
    if (mOnRelease) mOnRelease();
  }
  REF_COUNTED_NO_DESTRUCTOR(PoolLease);
};
}  // namespace

Result<IBuffer> BufferPool::take(bool block) noexcept {
  try {
    std::unique_lock<std::mutex> l(mLock);
    for (;;) {
      // a free buffer: one whose lease flag is clear
      for (size_t i = 0; i < mAll.size(); ++i) {
        if (!mLent[i]) {
          mLent[i] = true;
          mAll[i]->range()->clearRange();
          ref();
          auto* lease = new PoolLease(mAll[i].get(), [this, i]() {
            {
              std::lock_guard<std::mutex> g(mLock);
              mLent[i] = false;
            }
            mCv.notify_one();
            unref();
          });
          return makeRefResultNonNull<IBuffer>(lease);
        }
      }
      if (mAll.size() < mMax) {
        Ref<IBuffer> b;
        UNWRAP_OR_FWD_RESULT(b, mFactory->createBuffer(mSize));
        mAll.emplace_back(b.get());
        mLent.push_back(false);
        continue;
      }
      if (!block) return ERR_RESULT(Status_NotFound);
      mCv.wait(l);
    }
  }
  IF_CATCH_RETURN_RESULT;
}

// ---- util -------------------------------------------------------------------------------------------
Status BufferUtil::appendToBuffer(IBuffer* buffer, const void* src, size_t count,
                                  const IBufferCopier* copier) const noexcept {
  GS_REQUIRE_OR_RET_STATUS(count <= buffer->range()->remaining(), "append exceeds remaining capacity");
  FWD_IF_ERR(copier->copy(buffer->writePtr(), src, count));
  return buffer->range()->increaseEndOffset(count);
}

Status BufferUtil::readFromBuffer(void* dst, IBuffer* buffer, size_t count,
                                  const IBufferCopier* copier) const noexcept {
  GS_REQUIRE_OR_RET_STATUS(count <= buffer->range()->used(), "read exceeds used bytes");
  FWD_IF_ERR(copier->copy(dst, buffer->readPtr(), count));
  return buffer->range()->increaseOffset(count);
}

Status BufferUtil::moveFromBuffer(IBuffer* dst, IBuffer* src, size_t count,
                                  const IBufferCopier* copier) const noexcept {
  GS_REQUIRE_OR_RET_STATUS(count <= src->range()->used(), "move exceeds source used bytes");
  GS_REQUIRE_OR_RET_STATUS(count <= dst->range()->remaining(), "move exceeds destination capacity");
  FWD_IF_ERR(copier->copy(dst->writePtr(), src->readPtr(), count));
  FWD_IF_ERR(dst->range()->increaseEndOffset(count));
  return src->range()->increaseOffset(count);
}

}  // namespace gsdr_rt
