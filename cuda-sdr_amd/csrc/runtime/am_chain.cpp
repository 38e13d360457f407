// AM receive chain executor (include/gsdr/gsdr_amd.h, gsdrAmChain*): the C5 chain
// int8 IQ -> cf32 -> FC FIR -> AM -> FF FIR as one hipGraph per step.
//
// Stream semantics are those of the reference filters stepped one chunk at a time
// (Fir::getNumOutputElements / readOutput, Fir.cpp:141-279; QuadAmDemod.cpp:80-107;
// Int8ToFloat.cpp:80-100): the first chunk yields floor((L - T + 1) / D) RF outputs, after which
// every chunk of L samples yields exactly L / D, and the FIR keeps
//     r = T - 1 + ((L - T + 1) mod D)
// input samples between steps (Appendix A of SURVEY.md: same count rule, no wrap). The audio FIR
// behaves the same way on the AM stream (ra retained). With fixed r and ra every buffer of the
// steady state sits at a fixed address, so the step is captured once:
//
//   staging[p] = [ r history | L new ]  int8 IQ     (p = step parity; the carry goes to 1 - p)
//   am         = [ ra history | L/D new ] f32
//   graph(p):  gsdrInt8FirFCAmDemodFirFF(staging[p] -> am + ra,   (L/D RF outputs and, in the same
//                                        am -> audio)             launch, L/(D Da) audio outputs)
//              copy staging[p][L, L + r) -> staging[1-p][0, r)     (RF history)
//              copy am[La, La + ra) -> am[0, ra)                   (audio history)
//
// The first step has its own graph (input at staging[0] + r, AM written to the end of the window).
// Resident streams (gsdrAmChainStepResident) skip the staging window: the RF history is read in
// place in front of the caller's chunks and the whole multi-chunk segment is three launches.
// The chunk copy into staging[p] + r happens outside the graph (its source changes per step); in
// the pinned-ring mode it runs on a second stream, ordered by events against the step that last
// read staging[p], so it overlaps the previous step's compute.
#include <gsdr/gsdr_amd.h>
#include <gpusdrpipeline/GSLog.h>

#include <hip/hip_runtime.h>

#include <cstring>
#include <initializer_list>
#include <new>
#include <vector>

namespace {

#define AMC_TRY(expr__)                      \
  do {                                       \
    const hipError_t e__ = (expr__);         \
    if (e__ != hipSuccess) return e__;       \
  } while (false)

size_t firCount(size_t n, size_t T, size_t D) { return n < T ? 0 : (n - (T - 1)) / D; }  // Fir.cpp:178-186

}  // namespace

struct gsdrAmChainImpl {
  int32_t device = 0;
  size_t T = 0, D = 1, Ta = 0, Da = 1, L = 0, La = 0;
  size_t r = 0, ra = 0;    // retained input / AM samples between steps
  size_t n1 = 0, na1 = 0;  // first-step RF / audio output counts
  size_t naSteady = 0;
  float* taps = nullptr;
  float* audioTaps = nullptr;
  int8_t* staging[2] = {nullptr, nullptr};
  float* am = nullptr;
  float* audio = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t copyStream = nullptr;
  hipGraphExec_t first = nullptr;
  hipGraphExec_t steady[2] = {nullptr, nullptr};
  hipEvent_t readDone[2] = {nullptr, nullptr};  // staging[p] no longer read by the step that used it
  hipEvent_t copyDone[2] = {nullptr, nullptr};
  size_t steps = 0;
  // resident mode: [ra history | nChunks * La] AM window and its cached graph
  float* amBig = nullptr;
  size_t amBigChunks = 0;
  hipGraphExec_t resident = nullptr;
  const int8_t* resIn = nullptr;
  float* resOut = nullptr;
  size_t resChunks = 0;
  bool resFirst = false;
  // multi-chunk stepping (gsdrAmChainStepChunks): cached graphs of nChunks chunk steps over an AM
  // window [ra history | nChunks La], one per starting state (0 / 1 = the starting staging parity,
  // 2 = the stream's first step): with an odd nChunks the parity flips every call, so one cached
  // graph would be recaptured on every call
  hipGraphExec_t multi[3] = {nullptr, nullptr, nullptr};
  float* amMulti = nullptr;
  size_t amMultiChunks = 0;
  const int8_t* multiIn = nullptr;
  float* multiOut = nullptr;
  size_t multiChunks = 0;
  size_t captures = 0;  // graphs instantiated (creation's three + every recapture; diagnostics)
  // process-wide kernel settings baked into the cached graphs (kernel policy, FFT guard, WS spin
  // limit) at their capture
  uint64_t settings = 0;

  static uint64_t currentSettings() {
    const float g = gsdrAmdGetFftGuard();
    uint32_t gb = 0;
    std::memcpy(&gb, &g, sizeof gb);
    return ((uint64_t)gsdrAmdGetKernelPolicy() * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)gb << 32) ^
           (uint32_t)gsdrAmdGetWsSpinLimit();
  }
  // pinned ring
  size_t slots = 0;
  int8_t* hostIn = nullptr;
  float* hostOut = nullptr;
  int8_t* hostInDev = nullptr;  // the same slots as device pointers (hipHostGetDevicePointer)
  float* hostOutDev = nullptr;
  std::vector<hipEvent_t> slotDone;

  size_t nextOutputs() const { return steps == 0 ? na1 : naSteady; }

  hipError_t capture(hipGraphExec_t* exec, bool firstStep, int p) {
    hipGraph_t g = nullptr;
    AMC_TRY(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    hipError_t e = enqueueCompute(firstStep, p);
    hipError_t e2 = hipStreamEndCapture(stream, &g);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess) e = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    if (g != nullptr) (void)hipGraphDestroy(g);
    if (e == hipSuccess) ++captures;
    return e;
  }

  // Step entry: fail if the previous step's launch completed with a WS abort; recapture the
  // cached graphs when a process-wide kernel setting changed since their capture.
  hipError_t enter() {
    if (gsdrAmdWsAbortsPending(device) != 0) {  // rare: settle the count, then report it
      AMC_TRY(hipStreamSynchronize(copyStream));
      AMC_TRY(hipStreamSynchronize(stream));
      if (gsdrAmdWsTakeAborts(device) != 0) return hipErrorLaunchTimeOut;
    }
    const uint64_t now = currentSettings();
    if (now != settings) {
      AMC_TRY(hipStreamSynchronize(stream));
      for (hipGraphExec_t* g : {&first, &steady[0], &steady[1], &resident})
        if (*g != nullptr) {
          (void)hipGraphExecDestroy(*g);
          *g = nullptr;
        }
      dropMulti();
      settings = now;
      AMC_TRY(capture(&first, true, 0));
      AMC_TRY(capture(&steady[0], false, 0));
      AMC_TRY(capture(&steady[1], false, 1));
    }
    return hipSuccess;
  }

  void dropMulti() {
    for (auto& m : multi)
      if (m != nullptr) {
        (void)hipGraphExecDestroy(m);
        m = nullptr;
      }
  }

  hipError_t enqueueCompute(bool firstStep, int p) {
    const size_t amStart = firstStep ? ra + La - n1 : 0;  // first step: AM at the end of the window
    const int8_t* in = firstStep ? staging[p] + 2 * r : staging[p];
    const size_t nRf = firstStep ? n1 : La;
    // RF FIR + AM + audio FIR in one launch (the AM samples kept: the next step's audio history)
    AMC_TRY(gsdrInt8FirFCAmDemodFirFF(D, taps, T, in, nRf, am + amStart, firstStep ? 0 : ra, 1, Da, audioTaps, Ta,
                                      audio, firstStep ? na1 : naSteady, device, stream));
    AMC_TRY(hipMemcpyAsync(staging[1 - p], staging[p] + 2 * L, 2 * r, hipMemcpyDeviceToDevice, stream));
    AMC_TRY(hipMemcpyAsync(am, am + La, sizeof(float) * ra, hipMemcpyDeviceToDevice, stream));
    return hipSuccess;
  }

  hipGraphExec_t graphFor(int p) const { return steps == 0 ? first : steady[p]; }

  // RF outputs / audio outputs of a resident step of nChunks chunks
  size_t residentRf(size_t nChunks) const { return steps == 0 ? firCount(nChunks * L, T, D) : nChunks * La; }
  size_t residentAudio(size_t nChunks) const {
    const size_t nRf = residentRf(nChunks);
    return steps == 0 ? firCount(nRf, Ta, Da) : nChunks * naSteady;
  }

  hipError_t enqueueResident(const int8_t* in, size_t nChunks, float* out) {
    const size_t nRf = residentRf(nChunks);
    const size_t end = ra + nChunks * La;  // the AM window ends here in both cases
    const size_t amStart = steps == 0 ? end - nRf : 0;
    const int8_t* rfIn = steps == 0 ? in : in - 2 * r;
    AMC_TRY(gsdrInt8FirFCAmDemodFirFF(D, taps, T, rfIn, nRf, amBig + amStart, end - nRf - amStart, 1, Da, audioTaps,
                                      Ta, out, residentAudio(nChunks), device, stream));
    AMC_TRY(hipMemcpyAsync(amBig, amBig + end - ra, sizeof(float) * ra, hipMemcpyDeviceToDevice, stream));
    return hipSuccess;
  }

  // nChunks consecutive chunk steps from `in` (device, contiguous chunks), audio appended at `out`.
  // Each chunk is its own RF and audio launch, as stepping would be; only chunk 0 goes through the
  // staging window (behind the history carried from the previous step). Chunk i >= 1 reads its RF
  // history in place - the last r samples of chunk i - 1, right in front of it - and its AM
  // history in place in amMulti; the carries for the next step are copied out once at the end.
  hipError_t enqueueChunks(const int8_t* in, size_t nChunks, float* out, size_t startStep) {
    const bool first = startStep == 0;
    const int p0 = first ? 0 : (int)(startStep & 1);
    if (!first) {
      AMC_TRY(hipMemcpyAsync(staging[p0] + 2 * r, in, 2 * L, hipMemcpyDeviceToDevice, stream));
      AMC_TRY(hipMemcpyAsync(amMulti, am, sizeof(float) * ra, hipMemcpyDeviceToDevice, stream));
    }
    size_t pos = 0;
    for (size_t i = 0; i < nChunks; ++i) {
      const bool f = first && i == 0;
      const size_t nRf = f ? n1 : La;
      const int8_t* rfIn = f ? in : (i == 0 ? staging[p0] : in + 2 * (L * i - r));
      const size_t amEnd = ra + (i + 1) * La;  // chunk i's AM ends here (first step: n1 < La of it)
      // one launch per chunk: RF FIR + AM + the chunk's audio outputs (gsdrInt8FirFCAmDemodFirFF; r02
      // forked each chunk's audio FIR onto a second captured stream: 3.5x slower per chunk)
      const size_t na = f ? na1 : naSteady;
      const size_t amWin = f ? amEnd - n1 : amEnd - La - ra;
      AMC_TRY(gsdrInt8FirFCAmDemodFirFF(D, taps, T, rfIn, nRf, amMulti + amWin, amEnd - nRf - amWin, 1, Da, audioTaps,
                                        Ta, out + pos, na, device, stream));
      pos += na;
    }
    const int pn = (int)((startStep + nChunks) & 1);
    AMC_TRY(hipMemcpyAsync(staging[pn], in + 2 * (L * nChunks - r), 2 * r, hipMemcpyDeviceToDevice, stream));
    AMC_TRY(hipMemcpyAsync(am, amMulti + nChunks * La, sizeof(float) * ra, hipMemcpyDeviceToDevice, stream));
    return hipSuccess;
  }

  void release() {
    if (stream != nullptr) (void)hipStreamSynchronize(stream);
    if (copyStream != nullptr) (void)hipStreamSynchronize(copyStream);
    if (first) (void)hipGraphExecDestroy(first);
    for (auto& g : steady)
      if (g) (void)hipGraphExecDestroy(g);
    for (auto& ev : readDone)
      if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : copyDone)
      if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : slotDone)
      if (ev) (void)hipEventDestroy(ev);
    (void)hipFree(taps);
    (void)hipFree(audioTaps);
    (void)hipFree(staging[0]);
    (void)hipFree(staging[1]);
    (void)hipFree(am);
    (void)hipFree(amBig);
    if (resident) (void)hipGraphExecDestroy(resident);
    dropMulti();
    (void)hipFree(amMulti);
    (void)hipFree(audio);
    if (hostIn) (void)hipHostFree(hostIn);
    if (hostOut) (void)hipHostFree(hostOut);
    if (stream) (void)hipStreamDestroy(stream);
    if (copyStream) (void)hipStreamDestroy(copyStream);
  }
};

namespace {

struct DevicePush {  // the reference's CudaDevicePushPop (util/CudaDevicePushPop.h:27-79)
  int prev = -1;
  hipError_t err;
  explicit DevicePush(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DevicePush() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

hipError_t build(gsdrAmChainImpl* c, const gsdrAmChainConfig& cfg) {
  AMC_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  AMC_TRY(hipStreamCreateWithFlags(&c->copyStream, hipStreamNonBlocking));
  AMC_TRY(hipMalloc(&c->taps, sizeof(float) * c->T));
  AMC_TRY(hipMalloc(&c->audioTaps, sizeof(float) * c->Ta));
  AMC_TRY(hipMemcpy(c->taps, cfg.rfTaps, sizeof(float) * c->T, hipMemcpyHostToDevice));
  AMC_TRY(hipMemcpy(c->audioTaps, cfg.audioTaps, sizeof(float) * c->Ta, hipMemcpyHostToDevice));
  for (auto& s : c->staging) AMC_TRY(hipMalloc(&s, 2 * (c->r + c->L)));
  AMC_TRY(hipMalloc(&c->am, sizeof(float) * (c->ra + c->La)));
  AMC_TRY(hipMalloc(&c->audio, sizeof(float) * (c->na1 > c->naSteady ? c->na1 : c->naSteady)));
  for (auto& ev : c->readDone) AMC_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : c->copyDone) AMC_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  c->settings = gsdrAmChainImpl::currentSettings();
  if (c->slots > 0) {
    AMC_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->hostIn), 2 * c->L * c->slots, hipHostMallocDefault));
    AMC_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->hostOut), sizeof(float) * c->naSteady * c->slots,
                          hipHostMallocDefault));
    AMC_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hostInDev), c->hostIn, 0));
    AMC_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hostOutDev), c->hostOut, 0));
    c->slotDone.assign(c->slots, nullptr);
    for (auto& ev : c->slotDone) AMC_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }
  AMC_TRY(c->capture(&c->first, true, 0));
  AMC_TRY(c->capture(&c->steady[0], false, 0));
  AMC_TRY(c->capture(&c->steady[1], false, 1));
  return hipStreamSynchronize(c->stream);
}

}  // namespace

extern "C" {

hipError_t gsdrAmChainCreate(const gsdrAmChainConfig* cfg, int32_t device, gsdrAmChain* chainOut) {
  if (chainOut == nullptr) return hipErrorInvalidValue;
  *chainOut = nullptr;
  if (cfg == nullptr || cfg->rfTaps == nullptr || cfg->audioTaps == nullptr || cfg->rfTapCount == 0 ||
      cfg->audioTapCount == 0)
    return hipErrorInvalidValue;
  gsdrAmChainImpl* c = new (std::nothrow) gsdrAmChainImpl();
  if (c == nullptr) return hipErrorOutOfMemory;
  c->device = device;
  c->T = cfg->rfTapCount;
  c->D = cfg->rfDecimation < 1 ? 1 : cfg->rfDecimation;
  c->Ta = cfg->audioTapCount;
  c->Da = cfg->audioDecimation < 1 ? 1 : cfg->audioDecimation;
  c->L = cfg->chunkSamples;
  c->slots = cfg->hostSlots;
  const bool shapeOk = c->L >= c->T && c->L % (c->D * c->Da) == 0;
  if (shapeOk) {
    c->La = c->L / c->D;
    c->n1 = firCount(c->L, c->T, c->D);
    c->r = c->L - c->n1 * c->D;  // = T - 1 + ((L - T + 1) mod D)
    c->na1 = firCount(c->n1, c->Ta, c->Da);
    c->ra = c->n1 - c->na1 * c->Da;
    c->naSteady = c->La / c->Da;
  }
  // steady state: L/D RF and L/(D Da) audio outputs per step, disjoint history copies
  if (!shapeOk || c->na1 == 0 || c->r > c->L || c->ra > c->La ||
      firCount(c->r + c->L, c->T, c->D) != c->La || firCount(c->ra + c->La, c->Ta, c->Da) != c->naSteady) {
    delete c;
    return hipErrorInvalidValue;
  }
  DevicePush push(device);
  hipError_t e = push.err;
  if (e == hipSuccess) e = build(c, *cfg);
  if (e != hipSuccess) {
    c->release();
    delete c;
    return e;
  }
  *chainOut = c;
  return hipSuccess;
}

void gsdrAmChainDestroy(gsdrAmChain c) {
  if (c == nullptr) return;
  DevicePush push(c->device);
  c->release();
  delete c;
}

hipStream_t gsdrAmChainStream(gsdrAmChain c) { return c == nullptr ? nullptr : c->stream; }

size_t gsdrAmChainGraphCaptures(gsdrAmChain c) { return c == nullptr ? 0 : c->captures; }

size_t gsdrAmChainNextOutputCount(gsdrAmChain c) { return c == nullptr ? 0 : c->nextOutputs(); }

hipError_t gsdrAmChainStep(gsdrAmChain c, const int8_t* inputIq, float* output, size_t* outputCount) {
  if (c == nullptr || inputIq == nullptr || output == nullptr) return hipErrorInvalidValue;
  DevicePush push(c->device);
  AMC_TRY(push.err);
  AMC_TRY(c->enter());
  const int p = c->steps == 0 ? 0 : (int)(c->steps & 1);
  const size_t n = c->nextOutputs();
  AMC_TRY(hipMemcpyAsync(c->staging[p] + 2 * c->r, inputIq, 2 * c->L, hipMemcpyDeviceToDevice, c->stream));
  AMC_TRY(hipGraphLaunch(c->graphFor(p), c->stream));
  AMC_TRY(hipEventRecord(c->readDone[p], c->stream));
  AMC_TRY(hipMemcpyAsync(output, c->audio, sizeof(float) * n, hipMemcpyDeviceToDevice, c->stream));
  ++c->steps;
  if (outputCount != nullptr) *outputCount = n;
  return hipSuccess;
}

size_t gsdrAmChainChunksOutputCount(gsdrAmChain c, size_t nChunks) {
  if (c == nullptr || nChunks == 0) return 0;
  return c->steps == 0 ? c->na1 + (nChunks - 1) * c->naSteady : nChunks * c->naSteady;
}

hipError_t gsdrAmChainStepChunks(gsdrAmChain c, const int8_t* inputIq, size_t nChunks, float* output,
                                 size_t* outputCount) {
  if (c == nullptr || inputIq == nullptr || output == nullptr || nChunks == 0) return hipErrorInvalidValue;
  DevicePush push(c->device);
  AMC_TRY(push.err);
  AMC_TRY(c->enter());
  const size_t n = gsdrAmChainChunksOutputCount(c, nChunks);
  const int key = c->steps == 0 ? 2 : (int)(c->steps & 1);
  if (nChunks > c->amMultiChunks) {  // grow the AM window (outside any capture)
    AMC_TRY(hipStreamSynchronize(c->stream));
    c->dropMulti();
    (void)hipFree(c->amMulti);
    c->amMulti = nullptr;
    c->amMultiChunks = 0;
    AMC_TRY(hipMalloc(&c->amMulti, sizeof(float) * (c->ra + nChunks * c->La)));
    c->amMultiChunks = nChunks;
  }
  if (c->multiIn != inputIq || c->multiOut != output || c->multiChunks != nChunks) {
    // new buffers or chunk count: every cached start state is stale
    AMC_TRY(hipStreamSynchronize(c->stream));
    c->dropMulti();
    c->multiIn = inputIq;
    c->multiOut = output;
    c->multiChunks = nChunks;
  }
  if (c->multi[key] == nullptr) {
    hipGraph_t g = nullptr;
    AMC_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    hipError_t e = c->enqueueChunks(inputIq, nChunks, output, c->steps);
    const hipError_t e2 = hipStreamEndCapture(c->stream, &g);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess) e = hipGraphInstantiate(&c->multi[key], g, nullptr, nullptr, 0);
    if (g != nullptr) (void)hipGraphDestroy(g);
    AMC_TRY(e);
    ++c->captures;
  }
  AMC_TRY(hipGraphLaunch(c->multi[key], c->stream));
  // both staging parities were last read by this launch
  AMC_TRY(hipEventRecord(c->readDone[0], c->stream));
  AMC_TRY(hipEventRecord(c->readDone[1], c->stream));
  c->steps += nChunks;
  if (outputCount != nullptr) *outputCount = n;
  return hipSuccess;
}

int8_t* gsdrAmChainHostInputSlot(gsdrAmChain c, size_t slot) {
  return c == nullptr || slot >= c->slots ? nullptr : c->hostIn + 2 * c->L * slot;
}

const float* gsdrAmChainHostOutputSlot(gsdrAmChain c, size_t slot) {
  return c == nullptr || slot >= c->slots ? nullptr : c->hostOut + c->naSteady * slot;
}

hipError_t gsdrAmChainStepHost(gsdrAmChain c, size_t slot, size_t* outputCount) {
  if (c == nullptr || slot >= c->slots) return hipErrorInvalidValue;
  DevicePush push(c->device);
  AMC_TRY(push.err);
  AMC_TRY(c->enter());
  const int p = c->steps == 0 ? 0 : (int)(c->steps & 1);
  const size_t n = c->nextOutputs();
  // the H2D copy may start once the step that last read staging[p] is done with it
  AMC_TRY(hipStreamWaitEvent(c->copyStream, c->readDone[p], 0));
  // the copies as kernels on the mapped pinned slots: hipMemcpyAsync here blocked the host thread for
  // 7-10 ms in 10 of ~600 calls (r05 HIP API trace: the DMA itself 0.18 ms, issued at the end of the call)
  // (the copy kernel moves whole dwords from dword-aligned addresses: an odd r leaves the staging
  // destination 2 bytes off, an odd L the source slot and the byte count - the runtime copy then)
  if ((((2 * c->r) | (2 * c->L)) & 3) == 0)
    AMC_TRY(gsdrAmdCopyKernel(c->staging[p] + 2 * c->r, c->hostInDev + 2 * c->L * slot, 2 * c->L, c->copyStream));
  else
    AMC_TRY(hipMemcpyAsync(c->staging[p] + 2 * c->r, c->hostIn + 2 * c->L * slot, 2 * c->L, hipMemcpyHostToDevice,
                           c->copyStream));
  AMC_TRY(hipEventRecord(c->copyDone[p], c->copyStream));
  AMC_TRY(hipStreamWaitEvent(c->stream, c->copyDone[p], 0));
  AMC_TRY(hipGraphLaunch(c->graphFor(p), c->stream));
  AMC_TRY(hipEventRecord(c->readDone[p], c->stream));
  AMC_TRY(gsdrAmdCopyKernel(c->hostOutDev + c->naSteady * slot, c->audio, sizeof(float) * n, c->stream));
  AMC_TRY(hipEventRecord(c->slotDone[slot], c->stream));
  ++c->steps;
  if (outputCount != nullptr) *outputCount = n;
  return hipSuccess;
}

hipError_t gsdrAmChainWaitSlot(gsdrAmChain c, size_t slot) {
  if (c == nullptr || slot >= c->slots) return hipErrorInvalidValue;
  return hipEventSynchronize(c->slotDone[slot]);
}

size_t gsdrAmChainResidentOutputCount(gsdrAmChain c, size_t nChunks) {
  return c == nullptr ? 0 : c->residentAudio(nChunks);
}

hipError_t gsdrAmChainStepResident(gsdrAmChain c, const int8_t* inputIq, size_t nChunks, float* output,
                                   size_t* outputCount) {
  if (c == nullptr || inputIq == nullptr || output == nullptr || nChunks == 0) return hipErrorInvalidValue;
  DevicePush push(c->device);
  AMC_TRY(push.err);
  AMC_TRY(c->enter());
  if (nChunks > c->amBigChunks) {  // grow the AM window (outside any capture)
    AMC_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(c->amBig);
    c->amBig = nullptr;
    c->amBigChunks = 0;
    AMC_TRY(hipMalloc(&c->amBig, sizeof(float) * (c->ra + nChunks * c->La)));
    c->amBigChunks = nChunks;
    if (c->resident) (void)hipGraphExecDestroy(c->resident);
    c->resident = nullptr;
  }
  const bool firstStep = c->steps == 0;
  // The launch reads [inputIq - 2 r, inputIq + 2 L nChunks) after the first step (the RF history in
  // place) and [inputIq, ...) on it: both must lie inside inputIq's device allocation. A non-first step
  // handed a pointer with no room for its history in front read before the allocation and faulted the
  // GPU (r04, tools/exp/ws_abort_diag.py); it is now rejected with hipErrorInvalidValue instead.
  {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    const auto p = reinterpret_cast<uintptr_t>(inputIq);
    if (hipMemGetAddressRange(&base, &size, const_cast<int8_t*>(inputIq)) != hipSuccess || base == nullptr) {
      (void)hipGetLastError();
      gsloge("gsdrAmChainStepResident: inputIq is not device memory of this process");
      return hipErrorInvalidValue;
    }
    const auto lo = reinterpret_cast<uintptr_t>(base), hi = lo + size;
    const size_t before = firstStep ? 0 : 2 * c->r;
    if (p - lo < before || p + 2 * c->L * nChunks > hi) {
      gsloge("gsdrAmChainStepResident: the %s of this step lies outside inputIq's allocation (%zu bytes in front, "
             "%zu needed; %zu after, %zu needed)", p - lo < before ? "RF history in front" : "input",
             (size_t)(p - lo), before, (size_t)(hi - p), (size_t)(2 * c->L * nChunks));
      return hipErrorInvalidValue;
    }
  }
  if (c->resident == nullptr || c->resIn != inputIq || c->resOut != output || c->resChunks != nChunks ||
      c->resFirst != firstStep) {
    if (c->resident) (void)hipGraphExecDestroy(c->resident);
    c->resident = nullptr;
    hipGraph_t g = nullptr;
    AMC_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    hipError_t e = c->enqueueResident(inputIq, nChunks, output);
    const hipError_t e2 = hipStreamEndCapture(c->stream, &g);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess) e = hipGraphInstantiate(&c->resident, g, nullptr, nullptr, 0);
    if (g != nullptr) (void)hipGraphDestroy(g);
    AMC_TRY(e);
    ++c->captures;
    c->resIn = inputIq;
    c->resOut = output;
    c->resChunks = nChunks;
    c->resFirst = firstStep;
  }
  const size_t n = c->residentAudio(nChunks);
  AMC_TRY(hipGraphLaunch(c->resident, c->stream));
  // the AM history now sits at the front of amBig; the per-chunk window `am` is stale, so a later
  // per-chunk step would need a reset (documented in gsdr_amd.h)
  c->steps += nChunks;
  if (outputCount != nullptr) *outputCount = n;
  return hipSuccess;
}

hipError_t gsdrAmChainReset(gsdrAmChain c) {
  if (c == nullptr) return hipErrorInvalidValue;
  DevicePush push(c->device);
  AMC_TRY(push.err);
  AMC_TRY(hipStreamSynchronize(c->copyStream));
  AMC_TRY(hipStreamSynchronize(c->stream));
  c->steps = 0;
  return hipSuccess;
}

}  // extern "C"
