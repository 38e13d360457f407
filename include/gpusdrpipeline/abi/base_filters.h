/*
 * Helper base classes for filter implementations (reference filters/BaseSink.h:33-76,
 * BaseSource.h:24-35, BaseFilter.h:34-47). Source-compatible: filters derived from them must
 * be compiled against these headers.
 *
 * BaseSink keeps one growable device window per input port: requestBuffer() lends the unused
 * tail, commitBuffer() extends the used range, consumeInputBytesAndMoveUsedToStart() retires
 * consumed bytes. Unlike the reference (which relocates the retained bytes to offset 0 on every
 * consume, BaseSink.cpp:150-170), retired bytes are only compacted away when the next
 * requestBuffer() would not fit in the tail, and growth over-allocates 2x: the relocate copy is
 * amortised across steps instead of paid on every readOutput().
 */
#ifndef GPUSDRPIPELINE_ABI_BASE_FILTERS_H
#define GPUSDRPIPELINE_ABI_BASE_FILTERS_H

#include <gpusdrpipeline/abi/graph.h>

#include <vector>

class GS_PUBLIC BaseSink : public virtual Sink {
 public:
  struct InputPort {
    ConstRef<IRelocatableResizableBuffer> inputBuffer;
    bool bufferCheckedOut;
  };

  BaseSink() = delete;

  [[nodiscard]] Result<IBuffer> requestBuffer(size_t port, size_t numBytes) noexcept override;
  [[nodiscard]] Status commitBuffer(size_t port, size_t byteCount) noexcept override;

 protected:
  BaseSink(IRelocatableResizableBufferFactory* relocatableResizableBufferFactory,
           IBufferSliceFactory* slicedBufferFactory, size_t inputPortCount, IMemSet* memSet = nullptr);
  ~BaseSink() override = default;

  [[nodiscard]] Result<IBuffer> getPortInputBuffer(size_t port) noexcept;
  [[nodiscard]] Result<const IBuffer> getPortInputBuffer(size_t port) const noexcept;
  [[nodiscard]] bool inputPortsInitialized() const noexcept;

  /* Advance the port's used-range start by numBytes (the bytes are retired; the remaining
   * used bytes stay addressable through getPortInputBuffer()->readPtr()). */
  [[nodiscard]] Status consumeInputBytesAndMoveUsedToStart(size_t port, size_t numBytes) noexcept;

  /* MI355X extension (graph stepping, driver.h): folds every input window's placement (base
   * address, used range, capacity, checkout flag) into h. Non-virtual: no vtable change. */
  void foldWindowState(uint64_t& h) const noexcept;

 public:
  /* MI355X extension (graph replay, driver.h): the input windows and their checkout flags, so the
   * host state a captured step leaves behind can be saved and reinstated on replay. */
  [[nodiscard]] size_t inputWindowCount() const noexcept { return mInputPorts.size(); }
  [[nodiscard]] IRelocatableResizableBuffer* inputWindow(size_t port) const noexcept;
  [[nodiscard]] bool inputWindowCheckedOut(size_t port) const noexcept;
  void setInputWindowCheckedOut(size_t port, bool checkedOut) noexcept;

 private:
  const size_t mInputPortCount;
  ConstRef<IBufferSliceFactory> mSlicedBufferFactory;
  std::vector<InputPort> mInputPorts;
  ConstRef<IMemSet> mMemSet;
  ConstRef<IRelocatableResizableBufferFactory> mRelocatableResizableBufferFactory;

  [[nodiscard]] Status ensureInputPortsInit() noexcept;
};

class GS_PUBLIC BaseSource : public virtual Source {
 public:
  explicit BaseSource(std::vector<ImmutableRef<IBufferCopier>>&& outputPortBufferCopiers) noexcept;

  IBufferCopier* getOutputCopier(size_t port) noexcept override;

 protected:
  ~BaseSource() override = default;

 private:
  const std::vector<ImmutableRef<IBufferCopier>> mOutputPortBufferCopiers;
};

class GS_PUBLIC BaseFilter : public virtual Filter, public BaseSink, public BaseSource {
 public:
  BaseFilter() = delete;

 protected:
  BaseFilter(IRelocatableResizableBufferFactory* relocatableResizableBufferFactory,
             IBufferSliceFactory* slicedBufferFactory, size_t inputPortCount,
             std::vector<ImmutableRef<IBufferCopier>>&& outputPortBufferCopiers, IMemSet* memSet = nullptr) noexcept;
  ~BaseFilter() override = default;
};

#endif  // GPUSDRPIPELINE_ABI_BASE_FILTERS_H
