#include "filters.h"

#include <cstring>

#include <gsdr/conversion.h>
#include <gsdr/gsdr.h>
#include <gsdr/gsdr_amd.h>

#include <algorithm>
#include <cmath>

namespace gsdr_rt {

namespace {

Result<std::vector<ImmutableRef<IBufferCopier>>> deviceOutputCopiers(IFactories* f, ICudaCommandQueue* q) noexcept {
  try {
    Ref<IBufferCopier> d2d;
    UNWRAP_OR_FWD_RESULT(d2d, f->getCudaBufferCopierFactory()->createBufferCopier(q, hipMemcpyDeviceToDevice));
    std::vector<ImmutableRef<IBufferCopier>> v;
    v.emplace_back(d2d.get().get());
    return {.status = Status_Success, .value = std::move(v)};
  }
  IF_CATCH_RETURN_RESULT;
}

bool isFloatOrComplex(SampleType t) { return t == SampleType_Float || t == SampleType_FloatComplex; }

}  // namespace

size_t inputElementSize(SampleType t) noexcept {
  switch (t) {
    case SampleType_Float: return sizeof(float);
    case SampleType_FloatComplex: return 2 * sizeof(float);
    case SampleType_Int8Complex: return 2 * sizeof(int8_t);
    default: return 0;
  }
}

// ---- Fir (Fir.cpp:47-311) --------------------------------------------------------------------------
Result<Filter> Fir::create(SampleType tapType, SampleType elementType, size_t decimation, const float* taps,
                           size_t tapCount, ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  NON_NULL_PARAM_OR_RET(factories);
  // Supported: FF, FC, CC, CF and (Float taps, Int8Complex IQ input) -> cf32. The reference
  // accepts any pair and silently writes nothing for the others (Fir.cpp:229-269); here they
  // are rejected at creation.
  const bool ok = (isFloatOrComplex(tapType) && isFloatOrComplex(elementType)) ||
                  (tapType == SampleType_Float && elementType == SampleType_Int8Complex);
  GS_REQUIRE_OR_RET_RESULT_FMT(ok, "Unsupported FIR tap/element types [%u, %u]", tapType, elementType);

  Ref<IAllocator> allocator;
  Ref<IBufferCopier> h2d;
  Ref<IMemSet> memSet;
  Ref<IRelocatableResizableBufferFactory> windows;
  UNWRAP_OR_FWD_RESULT(allocator, factories->getCudaAllocatorFactory()->createCudaAllocator(queue, 32, false));
  UNWRAP_OR_FWD_RESULT(h2d, factories->getCudaBufferCopierFactory()->createBufferCopier(queue, hipMemcpyHostToDevice));
  UNWRAP_OR_FWD_RESULT(memSet, factories->getCudaMemSetFactory()->create(queue));
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, false));
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));

  auto* fir = new (std::nothrow) Fir(tapType, elementType, decimation, queue, allocator.get().get(),
                                     h2d.get().get(), windows.get().get(), factories->getBufferSliceFactory(),
                                     memSet.get().get(), std::move(copiers));
  NON_NULL_OR_RET(fir);
  const Status st = fir->setTaps(taps, tapCount);
  if (st != Status_Success) {
    fir->unref();  // floating object: unref at count 0 deletes (Fir.cpp:94-98)
    return ERR_RESULT(st);
  }
  return makeRefResultNonNull<Filter>(fir);
}

Fir::Fir(SampleType tapType, SampleType elementType, size_t decimation, ICudaCommandQueue* queue,
         IAllocator* allocator, IBufferCopier* h2d, IRelocatableResizableBufferFactory* windows,
         IBufferSliceFactory* slices, IMemSet* memSet, std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseFilter(windows, slices, 1, std::move(outputCopiers), memSet),
      mTapType(tapType),
      mElementType(elementType),
      mAllocator(allocator),
      mH2D(h2d),
      mDecimation(std::max<size_t>(1, decimation)),
      mQueue(queue),
      mInElem(inputElementSize(elementType)),
      mOutElem((tapType == SampleType_Float && elementType == SampleType_Float) ? sizeof(float)
                                                                                : 2 * sizeof(float)) {}

// Taps are applied in the order given (correlation). The allocation is sized for the tap TYPE
// (the reference allocates tapCount * 4 bytes and then copies 8 bytes per complex tap,
// Fir.cpp:126 vs :131-133).
Status Fir::setTaps(const float* taps, size_t tapCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(taps != nullptr || tapCount == 0, "taps must be non-null when tapCount > 0");
  const size_t bytes = tapCount * (mTapType == SampleType_FloatComplex ? 2 * sizeof(float) : sizeof(float));
  if (mTaps == nullptr || mTaps->capacity() < bytes) UNWRAP_OR_FWD_STATUS(mTaps, mAllocator->allocate(bytes));
  if (bytes > 0) FWD_IF_ERR(mH2D->copy(mTaps->data(), taps, bytes));
  mTapCount = tapCount;
  return Status_Success;
}

size_t Fir::availableInputs() const noexcept {
  if (!inputPortsInitialized()) return 0;
  Result<const IBuffer> in = getPortInputBuffer(0);
  if (in.status != Status_Success) return 0;
  return in.value->range()->used() / mInElem;
}

// Fir.cpp:141-186: floor((N - (T - 1)) / D), with the size_t wraps guarded (no output before
// T inputs are buffered; T = 0 never produces output).
size_t Fir::availableOutputs() const noexcept {
  const size_t n = availableInputs();
  if (mTapCount == 0 || n < mTapCount) return 0;
  return (n - (mTapCount - 1)) / mDecimation;
}

size_t Fir::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return availableOutputs() * mOutElem;
}

size_t Fir::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 32 * mOutElem;
}

Status Fir::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "Must have one output port");
  IBuffer* out = portOutputBuffers[0];
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  // partial reads never skip inputs (FirTests.cpp:96-221): write what fits, consume n*D
  const size_t n = std::min(availableOutputs(), out->range()->remaining() / mOutElem);
  if (n == 0) return Status_Success;

  const int32_t dev = mQueue->cudaDevice();
  hipStream_t s = mQueue->cudaStream();
  const void* x = in->readPtr();
  void* y = out->writePtr();
  hipError_t e;
  if (mElementType == SampleType_Int8Complex) {
    e = gsdrInt8FirFC(mDecimation, mTaps->as<float>(), mTapCount, static_cast<const int8_t*>(x),
                      static_cast<hipFloatComplex*>(y), n, dev, s);
  } else if (mTapType == SampleType_Float && mElementType == SampleType_Float) {
    e = gsdrFirFF(mDecimation, mTaps->as<float>(), mTapCount, static_cast<const float*>(x), static_cast<float*>(y), n,
                  dev, s);
  } else if (mTapType == SampleType_Float) {
    e = gsdrFirFC(mDecimation, mTaps->as<float>(), mTapCount, static_cast<const hipFloatComplex*>(x),
                  static_cast<hipFloatComplex*>(y), n, dev, s);
  } else if (mElementType == SampleType_FloatComplex) {
    e = gsdrFirCC(mDecimation, mTaps->as<hipFloatComplex>(), mTapCount, static_cast<const hipFloatComplex*>(x),
                  static_cast<hipFloatComplex*>(y), n, dev, s);
  } else {
    e = gsdrFirCF(mDecimation, mTaps->as<hipFloatComplex>(), mTapCount, static_cast<const float*>(x),
                  static_cast<hipFloatComplex*>(y), n, dev, s);
  }
  SAFE_HIP_OR_RET_STATUS(e);
  FWD_IF_ERR(out->range()->increaseEndOffset(n * mOutElem));
  return consumeInputBytesAndMoveUsedToStart(0, n * mDecimation * mInElem);
}

Status Fir::readOutputAm(IBuffer* out) noexcept {
  GS_REQUIRE_OR_RET_STATUS(out != nullptr && canFuseAm(), "Fir::readOutputAm needs real taps and an output");
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  const size_t n = std::min(availableOutputs(), out->range()->remaining() / sizeof(float));
  if (n == 0) return Status_Success;
  const int32_t dev = mQueue->cudaDevice();
  hipStream_t s = mQueue->cudaStream();
  hipError_t e;
  if (mElementType == SampleType_Int8Complex)
    e = gsdrInt8FirFCAmDemod(mDecimation, mTaps->as<float>(), mTapCount, in->readPtr<int8_t>(), out->writePtr<float>(),
                             n, dev, s);
  else
    e = gsdrFirFCAmDemod(mDecimation, mTaps->as<float>(), mTapCount, in->readPtr<hipFloatComplex>(),
                         out->writePtr<float>(), n, dev, s);
  SAFE_HIP_OR_RET_STATUS(e);
  FWD_IF_ERR(out->range()->increaseEndOffset(n * sizeof(float)));
  return consumeInputBytesAndMoveUsedToStart(0, n * mDecimation * mInElem);
}

// ---- QuadAmDemod (QuadAmDemod.cpp:31-109) ------------------------------------------------------------
Result<Filter> QuadAmDemod::create(ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  Ref<IRelocatableResizableBufferFactory> windows;
  Ref<IMemSet> memSet;
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, false));
  UNWRAP_OR_FWD_RESULT(memSet, factories->getCudaMemSetFactory()->create(queue));
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));
  return makeRefResultNonNull<Filter>(new (std::nothrow) QuadAmDemod(
      queue, windows.get().get(), factories->getBufferSliceFactory(), memSet.get().get(), std::move(copiers)));
}

QuadAmDemod::QuadAmDemod(ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows,
                         IBufferSliceFactory* slices, IMemSet* memSet,
                         std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseFilter(windows, slices, 1, std::move(outputCopiers), memSet), mQueue(queue) {}

size_t QuadAmDemod::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  Result<IBuffer> in = getPortInputBuffer(0);
  if (in.status != Status_Success) return 0;
  return in.value->range()->used() / (2 * sizeof(float)) * sizeof(float);
}

bool QuadAmDemod::inputEmpty() const noexcept {
  if (!inputPortsInitialized()) return true;
  Result<const IBuffer> in = getPortInputBuffer(0);
  return in.status == Status_Success && in.value->range()->used() == 0;
}

size_t QuadAmDemod::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 32 * sizeof(float);
}

Status QuadAmDemod::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "One output port is required");
  IBuffer* out = portOutputBuffers[0];
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  const size_t n = std::min(in->range()->used() / (2 * sizeof(float)), out->range()->remaining() / sizeof(float));
  if (n == 0) return Status_Success;
  SAFE_HIP_OR_RET_STATUS(gsdrQuadAmDemod(in->readPtr<hipFloatComplex>(), out->writePtr<float>(), n,
                                         mQueue->cudaDevice(), mQueue->cudaStream()));
  FWD_IF_ERR(out->range()->increaseEndOffset(n * sizeof(float)));
  return consumeInputBytesAndMoveUsedToStart(0, n * 2 * sizeof(float));
}

// ---- MultiplyCcc (Multiply.cpp:26-159) -------------------------------------------------------------------
Result<Filter> MultiplyCcc::create(ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  Ref<IRelocatableResizableBufferFactory> windows;
  Ref<IMemSet> memSet;
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, false));
  UNWRAP_OR_FWD_RESULT(memSet, factories->getCudaMemSetFactory()->create(queue));
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));
  return makeRefResultNonNull<Filter>(new (std::nothrow) MultiplyCcc(
      queue, windows.get().get(), factories->getBufferSliceFactory(), memSet.get().get(), std::move(copiers)));
}

MultiplyCcc::MultiplyCcc(ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows,
                         IBufferSliceFactory* slices, IMemSet* memSet,
                         std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseFilter(windows, slices, 2, std::move(outputCopiers), memSet), mQueue(queue) {}

// Multiply.cpp:63-76: the common prefix of both inputs
size_t MultiplyCcc::availableElements() const noexcept {
  if (!inputPortsInitialized()) return 0;
  Result<const IBuffer> a = getPortInputBuffer(0);
  Result<const IBuffer> b = getPortInputBuffer(1);
  if (a.status != Status_Success || b.status != Status_Success) return 0;
  return std::min(a.value->range()->used(), b.value->range()->used()) / sizeof(hipFloatComplex);
}

size_t MultiplyCcc::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Port [%zu] is out of range", port);
  return availableElements() * sizeof(hipFloatComplex);
}

size_t MultiplyCcc::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 32 * sizeof(hipFloatComplex);
}

// Multiply.cpp:82-121: ask the lagging port for the difference (capped at 100 MiB), the leading
// one for nothing; 8192 elements while both are empty.
size_t MultiplyCcc::preferredInputBufferSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port <= 1, 0, "Input port [%zu] is out of range", port);
  constexpr size_t kEmpty = 8192 * sizeof(hipFloatComplex);
  if (!inputPortsInitialized()) return kEmpty;
  Result<IBuffer> a = getPortInputBuffer(0);
  Result<IBuffer> b = getPortInputBuffer(1);
  if (a.status != Status_Success || b.status != Status_Success) return 0;
  const size_t u0 = a.value->range()->used(), u1 = b.value->range()->used();
  constexpr size_t kMax = 100 << 20;
  if (u0 == 0 && u1 == 0) return kEmpty;
  if (u0 >= u1) return port == 0 ? 0 : std::min(kMax, u0 - u1);
  return port == 0 ? std::min(kMax, u1 - u0) : 0;
}

Status MultiplyCcc::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "One output port is required");
  IBuffer* out = portOutputBuffers[0];
  const size_t n = std::min(availableElements(), out->range()->remaining() / sizeof(hipFloatComplex));
  if (n == 0) return Status_Success;
  Ref<IBuffer> a, b;
  UNWRAP_OR_FWD_STATUS(a, getPortInputBuffer(0));
  UNWRAP_OR_FWD_STATUS(b, getPortInputBuffer(1));
  // the reference ignores this status (Multiply.cpp:145, Appendix A): checked here
  SAFE_HIP_OR_RET_STATUS(gsdrMultiplyCC(a->readPtr<hipFloatComplex>(), b->readPtr<hipFloatComplex>(),
                                        out->writePtr<hipFloatComplex>(), n, mQueue->cudaDevice(),
                                        mQueue->cudaStream()));
  const size_t bytes = n * sizeof(hipFloatComplex);
  FWD_IF_ERR(out->range()->increaseEndOffset(bytes));
  FWD_IF_ERR(consumeInputBytesAndMoveUsedToStart(0, bytes));
  return consumeInputBytesAndMoveUsedToStart(1, bytes);
}

// ---- QuadFmDemod (QuadFmDemod.cpp:28-115) -----------------------------------------------------------------
Result<Filter> QuadFmDemod::create(float gain, ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  Ref<IRelocatableResizableBufferFactory> windows;
  Ref<IMemSet> memSet;
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, false));
  UNWRAP_OR_FWD_RESULT(memSet, factories->getCudaMemSetFactory()->create(queue));
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));
  return makeRefResultNonNull<Filter>(new (std::nothrow) QuadFmDemod(
      gain, queue, windows.get().get(), factories->getBufferSliceFactory(), memSet.get().get(), std::move(copiers)));
}

QuadFmDemod::QuadFmDemod(float gain, ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows,
                         IBufferSliceFactory* slices, IMemSet* memSet,
                         std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseFilter(windows, slices, 1, std::move(outputCopiers), memSet), mQueue(queue), mGain(gain) {}

size_t QuadFmDemod::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  Result<IBuffer> in = getPortInputBuffer(0);
  if (in.status != Status_Success) return 0;
  const size_t n = in.value->range()->used() / sizeof(hipFloatComplex);
  return (n == 0 ? 0 : n - 1) * sizeof(float);
}

size_t QuadFmDemod::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 32 * sizeof(float);
}

Status QuadFmDemod::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "One output port is required");
  IBuffer* out = portOutputBuffers[0];
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  const size_t avail = in->range()->used() / sizeof(hipFloatComplex);
  const size_t n = std::min(avail == 0 ? 0 : avail - 1, out->range()->remaining() / sizeof(float));
  if (n == 0) return Status_Success;
  SAFE_HIP_OR_RET_STATUS(gsdrQuadFmDemod(in->readPtr<hipFloatComplex>(), out->writePtr<float>(), mGain, n,
                                         mQueue->cudaDevice(), mQueue->cudaStream()));
  FWD_IF_ERR(out->range()->increaseEndOffset(n * sizeof(float)));
  return consumeInputBytesAndMoveUsedToStart(0, n * sizeof(hipFloatComplex));
}

// ---- Int8ToFloat (Int8ToFloat.cpp:32-102) ----------------------------------------------------------------
Result<Filter> Int8ToFloat::create(ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  Ref<IRelocatableResizableBufferFactory> windows;
  Ref<IMemSet> memSet;
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, false));
  UNWRAP_OR_FWD_RESULT(memSet, factories->getCudaMemSetFactory()->create(queue));
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));
  return makeRefResultNonNull<Filter>(new (std::nothrow) Int8ToFloat(
      queue, windows.get().get(), factories->getBufferSliceFactory(), memSet.get().get(), std::move(copiers)));
}

Int8ToFloat::Int8ToFloat(ICudaCommandQueue* queue, IRelocatableResizableBufferFactory* windows,
                         IBufferSliceFactory* slices, IMemSet* memSet,
                         std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseFilter(windows, slices, 1, std::move(outputCopiers), memSet), mQueue(queue) {}

size_t Int8ToFloat::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  Result<IBuffer> in = getPortInputBuffer(0);
  if (in.status != Status_Success) return 0;
  return in.value->range()->used() * sizeof(float);
}

size_t Int8ToFloat::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 32;
}

Status Int8ToFloat::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  // The reference requires portCount == 0 here (Int8ToFloat.cpp:81), which rejects every real
  // call; the evident intent (one output port) is implemented.
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "One output port is required");
  IBuffer* out = portOutputBuffers[0];
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  const size_t n = std::min(in->range()->used(), out->range()->remaining() / sizeof(float));
  if (n == 0) return Status_Success;
  SAFE_HIP_OR_RET_STATUS(gsdrInt8ToNormFloat(in->readPtr<int8_t>(), out->writePtr<float>(), n, mQueue->cudaDevice(),
                                             mQueue->cudaStream()));
  FWD_IF_ERR(out->range()->increaseEndOffset(n * sizeof(float)));
  return consumeInputBytesAndMoveUsedToStart(0, n);
}

// ---- Cosine sources (CosineSource.cpp:28-88, ComplexCosineSource.cpp:28-88) -------------------------------
Result<Source> CosineSource::create(bool complexOutput, float sampleRate, float frequency, ICudaCommandQueue* queue,
                                    IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  GS_REQUIRE_OR_RET_RESULT(sampleRate > 0.0f, "sampleRate must be positive");
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));
  return makeRefResultNonNull<Source>(
      new (std::nothrow) CosineSource(complexOutput, sampleRate, frequency, queue, std::move(copiers)));
}

CosineSource::CosineSource(bool complexOutput, float sampleRate, float frequency, ICudaCommandQueue* queue,
                           std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseSource(std::move(outputCopiers)),
      mComplex(complexOutput),
      mRadiansPerSample(static_cast<float>(2.0 * M_PI * frequency / sampleRate)),  // double, then float (:51)
      mQueue(queue) {}

size_t CosineSource::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return SIZE_MAX;  // infinite source
}

size_t CosineSource::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 32 * (mComplex ? 2 * sizeof(float) : sizeof(float));
}

// Fills the whole remaining capacity; the phase is carried (mod 2 pi) to the next call.
Status CosineSource::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "One output port is required");
  IBuffer* out = portOutputBuffers[0];
  const size_t elem = mComplex ? 2 * sizeof(float) : sizeof(float);
  const size_t n = out->range()->remaining() / elem;
  if (n == 0) return Status_Success;
  const float phiEnd = mPhi + static_cast<float>(n) * mRadiansPerSample;
  if (mComplex) {
    SAFE_HIP_OR_RET_STATUS(gsdrCosineC(mPhi, phiEnd, out->writePtr<hipFloatComplex>(), n, mQueue->cudaDevice(),
                                       mQueue->cudaStream()));
  } else {
    SAFE_HIP_OR_RET_STATUS(
        gsdrCosineF(mPhi, phiEnd, out->writePtr<float>(), n, mQueue->cudaDevice(), mQueue->cudaStream()));
  }
  mPhi = std::fmod(phiEnd, 2.0f * static_cast<float>(M_PI));
  return out->range()->increaseEndOffset(n * elem);
}

// ---- H2D / D2H staging (CudaMemcpyFilter.cpp:28-104) ---------------------------------------------------------
Result<Filter> HipMemcpyFilter::create(hipMemcpyKind kind, ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  const bool hostInput = kind == hipMemcpyHostToDevice || kind == hipMemcpyHostToHost;
  Ref<IRelocatableResizableBufferFactory> windows;
  Ref<IMemSet> memSet;
  Ref<IBufferCopier> copier;
  // a host-side input window is pinned (hipHostMalloc), so the copy is a true async DMA
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, hostInput));
  UNWRAP_OR_FWD_RESULT(memSet, factories->getCudaMemSetFactory()->create(queue));
  UNWRAP_OR_FWD_RESULT(copier, factories->getCudaBufferCopierFactory()->createBufferCopier(queue, kind));
  std::vector<ImmutableRef<IBufferCopier>> copiers;
  UNWRAP_MOVE_OR_FWD_RESULT(copiers, deviceOutputCopiers(factories, queue));
  return makeRefResultNonNull<Filter>(new (std::nothrow) HipMemcpyFilter(
      windows.get().get(), factories->getBufferSliceFactory(), memSet.get().get(), copier.get().get(), queue,
      std::move(copiers)));
}

HipMemcpyFilter::HipMemcpyFilter(IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
                                 IMemSet* memSet, IBufferCopier* copier, ICudaCommandQueue* queue,
                                 std::vector<ImmutableRef<IBufferCopier>>&& outputCopiers) noexcept
    : BaseFilter(windows, slices, 1, std::move(outputCopiers), memSet), mCopier(copier), mQueue(queue) {}

size_t HipMemcpyFilter::getOutputDataSize(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  Result<IBuffer> in = getPortInputBuffer(0);
  return in.status == Status_Success ? in.value->range()->used() : 0;
}

size_t HipMemcpyFilter::getOutputSizeAlignment(size_t port) noexcept {
  GS_REQUIRE_OR_RET_FMT(port == 0, 0, "Output port [%zu] is out of range", port);
  return 1;
}

Status HipMemcpyFilter::readOutput(IBuffer** portOutputBuffers, size_t portCount) noexcept {
  GS_REQUIRE_OR_RET_STATUS(portCount != 0 && portOutputBuffers != nullptr && portOutputBuffers[0] != nullptr,
                           "One output port is required");
  IBuffer* out = portOutputBuffers[0];
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  const size_t n = std::min(out->range()->remaining(), in->range()->used());
  if (n == 0) return Status_Success;
  FWD_IF_ERR(mCopier->copy(out->writePtr(), in->readPtr(), n));
  FWD_IF_ERR(out->range()->increaseEndOffset(n));
  return consumeInputBytesAndMoveUsedToStart(0, n);
}

// ---- device sink: the end of a chain whose output stays in HBM --------------------------------------
Result<Sink> DeviceSink::create(size_t preferredBytes, ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  Ref<IRelocatableResizableBufferFactory> windows;
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, false));
  return makeRefResultNonNull<Sink>(new (std::nothrow) DeviceSink(
      preferredBytes == 0 ? kDevicePreferredBytes : preferredBytes, windows.get().get(),
      factories->getBufferSliceFactory(), queue));
}

DeviceSink::DeviceSink(size_t preferredBytes, IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
                       ICudaCommandQueue* queue) noexcept
    : BaseSink(windows, slices, 1), mQueue(queue), mPreferred(preferredBytes) {}

Result<IBuffer> DeviceSink::requestBuffer(size_t port, size_t numBytes) noexcept {
  if (!inputPortsInitialized()) {  // creates the port windows on first use
    Ref<IBuffer> lazy;
    UNWRAP_OR_FWD_RESULT(lazy, getPortInputBuffer(port));
  }
  if (port < inputWindowCount() && !inputWindowCheckedOut(port)) {
    IRelocatableResizableBuffer* b = inputWindow(port);
    if (b != nullptr && b->range()->remaining() < numBytes) {
      if (b->range()->offset() != 0) FWD_IN_RESULT_IF_ERR(b->relocateUsedToStart());
      if (b->range()->remaining() < numBytes) FWD_IN_RESULT_IF_ERR(b->resize(b->range()->endOffset() + numBytes));
    }
  }
  return BaseSink::requestBuffer(port, numBytes);
}

Status DeviceSink::commitBuffer(size_t port, size_t byteCount) noexcept {
  FWD_IF_ERR(BaseSink::commitBuffer(port, byteCount));
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(port));
  return consumeInputBytesAndMoveUsedToStart(port, in->range()->used());
}

Result<Sink> HostEgressSink::create(ICudaCommandQueue* queue, IFactories* factories) noexcept {
  NON_NULL_PARAM_OR_RET(queue);
  Ref<IRelocatableResizableBufferFactory> windows;
  UNWRAP_OR_FWD_RESULT(windows, factories->createRelocatableCudaBufferFactory(queue, 32, true));  // pinned host
  return makeRefResultNonNull<Sink>(
      new (std::nothrow) HostEgressSink(windows.get().get(), factories->getBufferSliceFactory(), queue));
}

HostEgressSink::HostEgressSink(IRelocatableResizableBufferFactory* windows, IBufferSliceFactory* slices,
                               ICudaCommandQueue* queue) noexcept
    : BaseSink(windows, slices, 1), mQueue(queue), mWaiter(queue->cudaDevice(), queue->cudaStream()) {}

Result<IBuffer> HostEgressSink::requestBuffer(size_t port, size_t byteCount) noexcept {
  // the window would be compacted or grown by a stream-ordered copy: let the in-flight step land
  // and hand it over first, so no byte is read on the host while a copy may still move it
  bool fits = true;
  if (mInFlight != 0) {
    Ref<IBuffer> in;
    UNWRAP_OR_FWD_RESULT(in, getPortInputBuffer(port));
    fits = in->range()->remaining() >= byteCount;
  }
  if (!fits) {
    FWD_IN_RESULT_IF_ERR(mWaiter.waitAll());
    FWD_IN_RESULT_IF_ERR(deliver(0));
  }
  return BaseSink::requestBuffer(port, byteCount);
}

Status HostEgressSink::commitBuffer(size_t port, size_t byteCount) noexcept {
  FWD_IF_ERR(BaseSink::commitBuffer(port, byteCount));
  FWD_IF_ERR(mWaiter.recordNextAndWaitPrevious());  // everything before this commit is complete
  mInFlight = byteCount;
  return deliver(byteCount);
}

Status HostEgressSink::deliver(size_t keepInFlight) noexcept {
  Ref<IBuffer> in;
  UNWRAP_OR_FWD_STATUS(in, getPortInputBuffer(0));
  const size_t used = in->range()->used();
  const size_t ready = used > keepInFlight ? used - keepInFlight : 0;
  if (ready == 0) return Status_Success;
  try {
    // drop the consumed prefix once it is at least half the FIFO: a reader whose frame size does not
    // line up with the step size never empties it, and the FIFO must not grow with the stream
    if (mReadPos != 0 && 2 * mReadPos >= mFifo.size()) {
      mFifo.erase(mFifo.begin(), mFifo.begin() + (ptrdiff_t)mReadPos);
      mReadPos = 0;
    }
    const uint8_t* src = in->readPtr();
    mFifo.insert(mFifo.end(), src, src + ready);
  } catch (...) {
    return Status_OutOfMemory;
  }
  if (keepInFlight == 0) mInFlight = 0;
  return consumeInputBytesAndMoveUsedToStart(0, ready);
}

size_t HostEgressSink::read(void* dst, size_t capacity) noexcept {
  const size_t n = std::min(capacity, available());
  if (n != 0) memcpy(dst, mFifo.data() + mReadPos, n);
  mReadPos += n;
  return n;
}

Status HostEgressSink::flush() noexcept {
  FWD_IF_ERR(mWaiter.waitAll());
  return deliver(0);
}

}  // namespace gsdr_rt
