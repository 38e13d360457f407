// Hot-path filters over the gsdr gfx950 kernels (reference src/filters): Fir (Fir.cpp:32-311),
// QuadAmDemod (QuadAmDemod.cpp:28-109), Int8ToFloat (Int8ToFloat.cpp:30-102), CosineSource /
// ComplexCosineSource (CosineSource.cpp:28-88), and the H2D/D2H staging filter
// (CudaMemcpyFilter.cpp:28-104). Each readOutput() enqueues exactly one kernel (or copy) on the
// queue's stream and returns without synchronising, as in the reference.
#pragma once

#include "waiter.h"

#include <gpusdrpipeline/Factories.h>
#include <gpusdrpipeline/abi/base_filters.h>
#include <gpusdrpipeline/abi/errors.h>

#include "graph_state.h"

namespace gsdr_rt {

// Preferred input window of the device filters on MI355X. The reference asks for 1 MiB per step
// (Fir.cpp:311, QuadAmDemod.cpp:107), i.e. 131 072 cf32 samples: at C3's shape that is ~32 FFT
// blocks for 256 CUs x 8 waves, and every step pays its launches, so a driver-stepped chain ran at a
// fraction of the kernel rate. 256 MiB (33.5 M cf32 samples, several rounds of blocks on every CU)
// is cheap against 288 GB of HBM. The host staging filter keeps 1 MiB (PCIe transfers).
constexpr size_t kDevicePreferredBytes = size_t{256} << 20;

// Bytes per element of each SampleType on a filter's *input* side. Int8Complex is one I/Q
// pair (2 bytes); the reference's 1-byte size (Fir.cpp:34-45) never produced output.
size_t inputElementSize(SampleType t) noexcept;

class Fir final : public BaseFilter, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    h = (h ^ reinterpret_cast<uintptr_t>(mTaps.get() ? mTaps->data() : nullptr)) * 0x100000001B3ull + mTapCount;
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Filter> create(SampleType tapType, SampleType elementType, size_t decimation, const float* taps,
                               size_t tapCount, ICudaCommandQueue* queue, IFactories* factories) noexcept;

  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return kDevicePreferredBytes; }

  size_t decimation() const noexcept { return mDecimation; }
  size_t tapCount() const noexcept { return mTapCount; }

  // MI355X: the FIR and the AM envelope of a QuadAmDemod it feeds as ONE launch
  // (gsdrFirFCAmDemod / gsdrInt8FirFCAmDemod, bit-identical to gsdrFirFC + gsdrQuadAmDemod): the
  // envelope |y| goes straight into `out` (floats) and the cf32 outputs never touch HBM
  // (SteppingDriver fuses Fir -> QuadAmDemod edges, driver.cpp). Real taps only.
  bool canFuseAm() const noexcept {
    return mTapType == SampleType_Float &&
           (mElementType == SampleType_FloatComplex || mElementType == SampleType_Int8Complex);
  }
  size_t fusedAmOutputBytes() const noexcept { return availableOutputs() * sizeof(float); }
  Status readOutputAm(IBuffer* out) noexcept;
  hipStream_t stream() const noexcept { return mQueue->cudaStream(); }

 private:
  Fir(SampleType tapType, SampleType elementType, size_t decimation, ICudaCommandQueue* queue, IAllocator* allocator,
      IBufferCopier* h2d, IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices, IMemSet* memSet,
      std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  Status setTaps(const float* taps, size_t tapCount) noexcept;
  size_t availableInputs() const noexcept;
  size_t availableOutputs() const noexcept;

  const SampleType mTapType;
  const SampleType mElementType;
  ConstRef<IAllocator> mAllocator;
  ConstRef<IBufferCopier> mH2D;
  const size_t mDecimation;
  Ref<IMemory> mTaps;
  size_t mTapCount = 0;
  ConstRef<ICudaCommandQueue> mQueue;
  const size_t mInElem;
  const size_t mOutElem;

  REF_COUNTED(Fir);
};

class QuadAmDemod final : public BaseFilter, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Filter> create(ICudaCommandQueue* queue, IFactories* factories) noexcept;
  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return kDevicePreferredBytes; }
  bool inputEmpty() const noexcept;  // no cf32 left in the window (fusion keeps it empty)
  hipStream_t stream() const noexcept { return mQueue->cudaStream(); }

 private:
  QuadAmDemod(ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
              IMemSet* memSet, std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  ConstRef<ICudaCommandQueue> mQueue;
  REF_COUNTED(QuadAmDemod);
};

// Two-input complex multiply (Multiply.cpp:26-159): the frequency shifter's mixer when port 1 is
// fed by a ComplexCosine source.
class MultiplyCcc final : public BaseFilter, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Filter> create(ICudaCommandQueue* queue, IFactories* factories) noexcept;
  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final;

 private:
  MultiplyCcc(ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
              IMemSet* memSet, std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  size_t availableElements() const noexcept;
  ConstRef<ICudaCommandQueue> mQueue;
  REF_COUNTED(MultiplyCcc);
};

// Quadrature FM discriminator (QuadFmDemod.cpp:28-115): n inputs -> n - 1 outputs, the last input
// kept for the next call.
class QuadFmDemod final : public BaseFilter, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Filter> create(float gain, ICudaCommandQueue* queue, IFactories* factories) noexcept;
  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return kDevicePreferredBytes; }

 private:
  QuadFmDemod(float gain, ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows,
              IBufferSliceFactory* slices, IMemSet* memSet,
              std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  ConstRef<ICudaCommandQueue> mQueue;
  const float mGain;
  REF_COUNTED(QuadFmDemod);
};

class Int8ToFloat final : public BaseFilter, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Filter> create(ICudaCommandQueue* queue, IFactories* factories) noexcept;
  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return kDevicePreferredBytes; }

 private:
  Int8ToFloat(ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
              IMemSet* memSet, std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  ConstRef<ICudaCommandQueue> mQueue;
  REF_COUNTED(Int8ToFloat);
};

// Infinite phase-continuous tone (cos for Float, exp(j phi) for FloatComplex).
class CosineSource final : public BaseSource, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t&) const noexcept final { return false; }  // the phase argument advances
  bool saveStepState(GraphNodeState&) const noexcept final { return false; }
  Status restoreStepState(const GraphNodeState&) noexcept final { return Status_InvalidState; }

  static Result<Source> create(bool complexOutput, float sampleRate, float frequency, ICudaCommandQueue* queue,
                               IFactories* factories) noexcept;
  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final;

 private:
  CosineSource(bool complexOutput, float sampleRate, float frequency, ICudaCommandQueue* queue,
               std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  const bool mComplex;
  const float mRadiansPerSample;
  ConstRef<ICudaCommandQueue> mQueue;
  float mPhi = 0.0f;
  REF_COUNTED(CosineSource);
};

class HipMemcpyFilter final : public BaseFilter, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Filter> create(hipMemcpyKind kind, ICudaCommandQueue* queue, IFactories* factories) noexcept;
  size_t getOutputDataSize(size_t port) noexcept final;
  size_t getOutputSizeAlignment(size_t port) noexcept final;
  Status readOutput(IBuffer** portOutputBuffers, size_t numPorts) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return 1 << 20; }

 private:
  HipMemcpyFilter(IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices, IMemSet* memSet,
                  IBufferCopier* copier, ICudaCommandQueue* queue,
                  std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept;
  ConstRef<IBufferCopier> mCopier;
  ConstRef<ICudaCommandQueue> mQueue;
  REF_COUNTED(HipMemcpyFilter);
};

// A device-memory sink that retires every committed byte (the consumer of a benchmarked chain, or
// any graph tail whose output is not read back): its window never grows past one step.
class DeviceSink final : public BaseSink, public IGraphStepState {
 public:
  hipStream_t graphStream() const noexcept final { return mQueue->cudaStream(); }
  bool graphState(uint64_t& h) const noexcept final {
    foldWindowState(h);
    h = (h ^ mPreferred) * 0x100000001B3ull;
    return true;
  }
  bool saveStepState(GraphNodeState& out) const noexcept final { return saveSinkWindows(*this, out); }
  Status restoreStepState(const GraphNodeState& in) noexcept final { return restoreSinkWindows(*this, in); }
  static Result<Sink> create(size_t preferredBytes, ICudaCommandQueue* queue, IFactories* factories) noexcept;
  // grows the window to exactly the request, as the reference's BaseSink does (BaseSink.cpp:75-77):
  // the window never holds history (every commit is consumed), so the 2x headroom BaseSink takes
  // for appending steps buys nothing here and would let a step run past the preferred size
  Result<IBuffer> requestBuffer(size_t port, size_t numBytes) noexcept final;
  Status commitBuffer(size_t port, size_t byteCount) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return mPreferred; }

 private:
  DeviceSink(size_t preferredBytes, IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
             ICudaCommandQueue* queue) noexcept;
  ConstRef<ICudaCommandQueue> mQueue;
  const size_t mPreferred;
  REF_COUNTED(DeviceSink);
};

// Egress: the host end of a chain (reference AacFileWriter.cpp:267-280 minus the codec, with the
// Waiter of Waiter.cpp:34-50). The input window is pinned host memory, so the upstream kernel
// writes its output straight into it. commitBuffer records an event after the committed work and
// waits for the PREVIOUS commit's event: one step stays in flight (the stream stays full) while
// every byte committed before it is moved to the host FIFO that read() drains. flush() waits for
// the in-flight step and delivers it too.
class HostEgressSink final : public BaseSink {
 public:
  static Result<Sink> create(ICudaCommandQueue* queue, IFactories* factories) noexcept;
  Result<IBuffer> requestBuffer(size_t port, size_t byteCount) noexcept final;
  Status commitBuffer(size_t port, size_t byteCount) noexcept final;
  size_t preferredInputBufferSize(size_t port) noexcept final { return 1 << 20; }

  size_t available() const noexcept { return mFifo.size() - mReadPos; }
  size_t read(void* dst, size_t capacity) noexcept;
  Status flush() noexcept;

 private:
  HostEgressSink(IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
                 ICudaCommandQueue* queue) noexcept;
  Status deliver(size_t keepInFlight) noexcept;
  ConstRef<ICudaCommandQueue> mQueue;
  Waiter mWaiter;
  size_t mInFlight = 0;  // bytes of the last commit, possibly still being written
  std::vector<uint8_t> mFifo;
  size_t mReadPos = 0;
  REF_COUNTED(HostEgressSink);
};

}  // namespace gsdr_rt
