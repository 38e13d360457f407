/*
 * gsdr_amd.h - MI355X-only extensions to the gsdr kernel ABI.
 *
 * Fused chain kernels for the FIR -> QuadAmDemod hot path (BASELINE.json north star).
 * They compute exactly what the corresponding chain of reference entry points computes
 * (same arithmetic per stage, intermediates kept on chip instead of in HBM):
 *
 *   gsdrInt8FirFC          == gsdrInt8ToNormFloat -> gsdrFirFC
 *   gsdrInt8FirFCAmDemod   == gsdrInt8ToNormFloat -> gsdrFirFC -> gsdrQuadAmDemod
 *   gsdrFirFCAmDemod       == gsdrFirFC -> gsdrQuadAmDemod
 *   gsdrFirCCAmDemod       == gsdrFirCC -> gsdrQuadAmDemod
 *
 * `inputIq` is interleaved int8 I,Q (2 bytes per complex sample); `outputCount` counts
 * FIR outputs exactly as in gsdr.h, so the caller supplies
 * (outputCount - 1) * decimation + tapCount complex input samples.
 */
#ifndef GSDR_GSDR_AMD_H
#define GSDR_GSDR_AMD_H

#include <gsdr/gsdr.h>

#ifdef __cplusplus
extern "C" {
#endif

GSDR_API hipError_t gsdrInt8FirFC(size_t decimation, const float* taps, size_t tapCount, const int8_t* inputIq,
                                  hipFloatComplex* output, size_t outputCount, int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrInt8FirFCAmDemod(size_t decimation, const float* taps, size_t tapCount,
                                         const int8_t* inputIq, float* output, size_t outputCount, int32_t device,
                                         hipStream_t stream);
GSDR_API hipError_t gsdrFirFCAmDemod(size_t decimation, const float* taps, size_t tapCount,
                                     const hipFloatComplex* input, float* output, size_t outputCount, int32_t device,
                                     hipStream_t stream);
GSDR_API hipError_t gsdrFirCCAmDemod(size_t decimation, const hipFloatComplex* taps, size_t tapCount,
                                     const hipFloatComplex* input, float* output, size_t outputCount, int32_t device,
                                     hipStream_t stream);

/*
 * The C5 receive chain in ONE launch: int8 IQ -> FC FIR (taps, decimation) -> AM -> FF audio FIR
 * (audioTaps, audioDecimation). amWindow = [amHistory AM samples carried from before | rfCount new];
 * the call computes
 *     gsdrInt8FirFCAmDemod(decimation, taps, tapCount, inputIq, amWindow + amHistory, rfCount)
 *     gsdrFirFF(audioDecimation, audioTaps, audioTapCount, amWindow, audioOut, audioCount)
 * with (audioCount - 1) audioDecimation + audioTapCount <= amHistory + rfCount. On the
 * wave-specialised int8 matrix-core kernel (the C5 RF shape) the AM samples stay on chip: each
 * tile's AM goes to an LDS ring and the kernel's producer waves run the audio FIR from it (<= 256
 * audio taps; each audio output a 64-lane sum of 4-tap partials - the same terms as gsdrFirFF in
 * another order). storeAm = 0 leaves amWindow[amHistory..] unspecified (not written by the fused
 * kernel; other shapes use it as the intermediate); 1 stores the AM samples there as the first call
 * would. Other shapes and policies run the two calls.
 */
GSDR_API hipError_t gsdrInt8FirFCAmDemodFirFF(size_t decimation, const float* taps, size_t tapCount,
                                              const int8_t* inputIq, size_t rfCount, float* amWindow,
                                              size_t amHistory, int storeAm, size_t audioDecimation,
                                              const float* audioTaps, size_t audioTapCount, float* audioOut,
                                              size_t audioCount, int32_t device, hipStream_t stream);

/*
 * Streaming form of gsdrInt8FirFCAmDemod: the same outputs, and the history the next call needs
 * (input samples [outputCount * decimation, (outputCount - 1) * decimation + tapCount), i.e. the
 * last tapCount - decimation samples) is copied to carryIq in the same launch. carryIq may alias
 * the start of inputIq - the in-place layout [history | new samples] of a streaming FIR, where the
 * next block of samples is then written right behind the carried history. It must not alias
 * any other part of inputIq or the output.
 */
GSDR_API hipError_t gsdrInt8FirFCAmDemodCarry(size_t decimation, const float* taps, size_t tapCount,
                                              const int8_t* inputIq, float* output, size_t outputCount,
                                              int8_t* carryIq, int32_t device, hipStream_t stream);

/*
 * Frequency shifter fused into the FIR input load (the reference's
 * ComplexCosineSource -> MultiplyCcc -> Fir front end, RfToPcmAudioFactory.cpp:218-235): input
 * sample n (n = 0 at `input`) is multiplied by exp(j theta(n)) before the FIR,
 *     theta(n) = phase0 + n * radiansPerSample,
 * reduced exactly modulo 2 pi (64-bit fixed-point cycle fractions) and then evaluated in float
 * (sincosf); the product is the gsdrMultiplyCC expression. A streaming caller advances phase0 by
 * consumed * radiansPerSample (mod 2 pi) between calls. No tone is materialised in HBM.
 */
GSDR_API hipError_t gsdrMixFirFC(size_t decimation, const float* taps, size_t tapCount, const hipFloatComplex* input,
                                 double phase0, double radiansPerSample, hipFloatComplex* output, size_t outputCount,
                                 int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrMixFirFCAmDemod(size_t decimation, const float* taps, size_t tapCount,
                                        const hipFloatComplex* input, double phase0, double radiansPerSample,
                                        float* output, size_t outputCount, int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrInt8MixFirFC(size_t decimation, const float* taps, size_t tapCount, const int8_t* inputIq,
                                     double phase0, double radiansPerSample, hipFloatComplex* output,
                                     size_t outputCount, int32_t device, hipStream_t stream);
GSDR_API hipError_t gsdrInt8MixFirFCAmDemod(size_t decimation, const float* taps, size_t tapCount,
                                            const int8_t* inputIq, double phase0, double radiansPerSample,
                                            float* output, size_t outputCount, int32_t device, hipStream_t stream);

/*
 * Fused FM front: frequency shift (as gsdrMixFirFC) -> low-pass FIR, decimate ->
 * FM discriminator (the gsdrQuadFmDemod expression gain * arg(y[k+1] conj(y[k]))) in one kernel:
 * output k uses FIR outputs k and k + 1, so the caller supplies outputCount * decimation + tapCount
 * input samples (outputCount + 1 FIR outputs). A streaming caller carries the last FIR output's
 * window like any FIR (consume outputCount * decimation samples); the discriminator's "previous
 * sample" is the recomputed FIR output k, so nothing else is carried. Equals gsdrMixFirFC followed
 * by gsdrQuadFmDemod bit for bit.
 */
GSDR_API hipError_t gsdrMixFirFCFmDemod(size_t decimation, const float* taps, size_t tapCount,
                                        const hipFloatComplex* input, double phase0, double radiansPerSample,
                                        float gain, float* output, size_t outputCount, int32_t device,
                                        hipStream_t stream);
GSDR_API hipError_t gsdrInt8MixFirFCFmDemod(size_t decimation, const float* taps, size_t tapCount,
                                            const int8_t* inputIq, double phase0, double radiansPerSample, float gain,
                                            float* output, size_t outputCount, int32_t device, hipStream_t stream);
/*
 * The reference's fused FM front gsdrFmDemod (call site src/applications/fm_simpletest.cpp:400-413;
 * gsdr itself is not vendored, so argument types follow that call site): sample n of `input` is
 * mixed by exp(j 2 pi (tuned - channel) (firstSampleOffset + n) / rfSampleRate), low-passed and
 * decimated by rfLowPassDecimation, and discriminated with the QuadDemodFactory gain
 * (rfSampleRate / D) / (2 pi channelFmDeviation 5) (QuadDemodFactory.h:108-110).
 */
GSDR_API hipError_t gsdrFmDemod(size_t rfSampleRate, float tunedFrequency, float channelFrequency,
                                float channelFmDeviation, size_t rfLowPassDecimation, size_t firstSampleOffset,
                                const float* taps, size_t tapCount, const hipFloatComplex* input, float* output,
                                size_t outputCount, int32_t device, hipStream_t stream);

/*
 * Deterministic synthetic sources for the benchmark configurations.
 * Sample n (absolute stream index firstSample + i) depends only on (seed, n), so a
 * time-sharded stream is generated shard by shard with no communication.
 *
 * C2-style HackRF IQ (int8, 2 bytes per sample):
 *   s[n] = 100 (1 + 0.5 cos(2 pi fAm n / fs)) exp(j 2 pi fCarrier n / fs) + u[n],
 *   u = uniform in [-3, 3) per component from splitmix64(seed ^ (2n + c)),
 *   rounded half away from zero, clipped to [-127, 127].
 * C3-style wideband cf32:
 *   x[n] = exp(j 2 pi f1 n) + 0.5 exp(j 2 pi f2 n) + 0.01 (u_r + j u_i),  u in [-1, 1),
 *   f1, f2 in cycles per sample.
 * Phases are reduced in double precision (n mod period) before the float trig.
 */
/*
 * Kernel-selection policy (process-wide; default 0). GSDR_POLICY_NO_MFMA routes every FIR through
 * the fp32 VALU direct-form kernels (no matrix-core and no FFT kernel; A/B comparisons).
 */
#define GSDR_POLICY_NO_MFMA 1u
/* cf32 x real taps on the bf16 x 3 split (6 products) instead of f16 x 2 with per-tile scale. */
#define GSDR_POLICY_CF_BF16 2u
/* Decimating MFMA FIRs on the barrier-synchronous kernels instead of the wave-specialised
 * (producer / consumer) ones. */
#define GSDR_POLICY_NO_WS 4u
/* Long real-tap FIRs (T >= 256, D in {2,4,6,8,10}) on the matrix-core / VALU direct forms instead of
 * the FFT fast convolution (polyphase overlap-save, fp32). */
#define GSDR_POLICY_NO_FFT 8u
/* The FFT fast convolution wherever it is eligible: int8 IQ input even where the int8 MFMA kernels
 * apply (by default they do: faster for int8 at the C5 shape), and cf32 launches below 2^24 input
 * samples, which by default take the MFMA kernel (r06: faster for a live stream's small steps); A/B
 * comparisons and tests of the FFT path at small sizes. */
#define GSDR_POLICY_PREFER_FFT 16u
/* int8 IQ decimating MFMA FIRs (and the fused C5 chain) on the 8-way split-K wave-specialised kernel of
 * r01-r04 instead of the 4-way one (r05: one consumer wave per SIMD); A/B
 * comparisons. (32u is taken by experimental builds.) */
#define GSDR_POLICY_I8_WS8 64u
GSDR_API void gsdrAmdSetKernelPolicy(uint32_t flags);
/* The kernel family the FC FIR entry points pick for this shape under the current policy:
 * "fft", "i8-mfma", "i8-dec-mfma", "cf-mfma" or "valu" (diagnostics / benchmark labels). */
GSDR_API const char* gsdrAmdFirKernelClass(int int8Iq, size_t tapCount, size_t decimation, const void* input);
GSDR_API uint32_t gsdrAmdGetKernelPolicy(void);
/* FFT FIR accuracy guard: each FFT block is cut into segments of >= 16 consecutive samples; a block
 * whose loudest segment's level (root of its energy sum |x|^2) exceeds `ratio` times its quietest
 * segment's (compared on energies: hi <= ratio^2 lo), or that holds inf/NaN, is computed in the
 * direct fp32 form. Default 8; 0 forces the direct form everywhere (tests). */
GSDR_API void gsdrAmdSetFftGuard(float ratio);
GSDR_API float gsdrAmdGetFftGuard(void);
/* Diagnostics: blocks the FFT FIR computed in the direct form on `device` since the last reset
 * (synchronises the device; reset != 0 zeroes the counter). */
GSDR_API hipError_t gsdrAmdFftDirectBlocks(int32_t device, uint64_t* count, int reset);
/* Wave-specialised (producer / consumer) MFMA FIR kernels: every hand-off wait gives up after
 * `microseconds` of wall clock (s_memrealtime; default 2 000 000 = 2 s; 0: at the first poll that finds
 * the hand-off pending - tests), releases all other waits so the grid drains, and counts the abort in a
 * host-visible word. (Through r05 the limit counted s_sleep polls, whose duration depends on whatever
 * else runs on the CU.) Such a launch's outputs are undefined; the
 * next gsdr* call that launches a wave-specialised kernel on that device returns
 * hipErrorLaunchTimeOut (and clears the count). gsdrAmdWsAborts synchronises `device` and reads
 * the count (reset != 0 clears it). */
GSDR_API void gsdrAmdSetWsSpinLimit(int32_t microseconds);
GSDR_API int32_t gsdrAmdGetWsSpinLimit(void);
GSDR_API hipError_t gsdrAmdWsAborts(int32_t device, uint64_t* count, int reset);
/* The count is per DEVICE, not per stream or executor: an abort raised by a launch of another stream
 * or chain on the same device is reported by whichever wave-specialised call (or executor step)
 * looks next, and cleared there.
 * The same count WITHOUT synchronising: Pending peeks (no clear), Take reads and clears. For graph
 * executors: when Pending is nonzero they synchronise their stream, then Take, then fail the step.
 * The eager entry points do the same (device-wide), so a caller that synchronises after a launch
 * gets an abort reported by its next call, and the common case costs no API call. */
GSDR_API uint32_t gsdrAmdWsTakeAborts(int32_t device);
GSDR_API uint32_t gsdrAmdWsAbortsPending(int32_t device);
/* Build provenance: 16 hex digits of the sha256 over the sources this library was built from
 * (tools/source_hash.py: kernels, runtime, C API, public headers, Makefile). A library that does not
 * match the tree it is tested with fails tests/test_abi_exports.py. */
GSDR_API const char* gsdrAmdBuildId(void);
/* The compiler that built it: HIP and clang version numbers (not part of the id, r06). */
GSDR_API const char* gsdrAmdBuildCompiler(void);
/* Diagnostics: HBM bandwidth probe over `bytes` (16-byte aligned device buffers): mode 0 streams
 * `input` (float4 loads, one sum per thread; `output` untouched for finite data), mode 1 copies it to
 * `output`. The bench times it to report the roofline against measured bandwidth as well as spec. */
GSDR_API hipError_t gsdrAmdHbmProbe(const void* input, void* output, size_t bytes, int32_t mode, int32_t device,
                                    hipStream_t stream);
/* Tests: fill the LDS of every CU of `device` with the 32-bit `pattern` (one workgroup of the whole
 * LDS per slot, 4 per CU) on `stream`, so that a later kernel reading LDS it never wrote sees it. */
GSDR_API hipError_t gsdrAmdPoisonLds(uint32_t pattern, int32_t device, hipStream_t stream);
/* A copy as a kernel on `stream`: `src` / `dst` device memory or mapped pinned host memory (device
 * pointers from hipHostGetDevicePointer), 4-byte aligned, `bytes` a multiple of 4 (16-byte loads when
 * `src` and `bytes` are 16-byte aligned). The host-fed chain moves its chunks with it: hipMemcpyAsync
 * between pinned host slots and the device blocked the host thread 7-10 ms in 10 of ~600 calls (r05
 * HIP API trace), a kernel launch never does. hipErrorInvalidValue on misalignment. */
GSDR_API hipError_t gsdrAmdCopyKernel(void* dst, const void* src, size_t bytes, hipStream_t stream);

GSDR_API hipError_t gsdrSynthIqInt8(uint64_t seed, double sampleRate, double amToneHz, double carrierHz,
                                    uint64_t firstSample, int8_t* outputIq, size_t numSamples, int32_t device,
                                    hipStream_t stream);
GSDR_API hipError_t gsdrSynthWidebandCf32(uint64_t seed, double f1, double f2Cycles, uint64_t firstSample,
                                          hipFloatComplex* output, size_t numSamples, int32_t device,
                                          hipStream_t stream);

/*
 * AM receive chain executor (C5: int8 IQ -> cf32 -> FC FIR (rf taps, rf decimation) -> AM ->
 * FF FIR (audio taps, audio decimation)), stepping fixed chunks of `chunkSamples` IQ samples.
 *
 * Output is exactly what the reference filters chained by a SteppingDriver produce from the same
 * stream (Fir count rule Fir.cpp:178-186 at both FIRs; the first step emits fewer samples), but
 * the steady-state step is ONE hipGraph launch (FIR+AM kernel, history carries, audio FIR) captured
 * at creation, with every buffer at a fixed address: a [history | chunk] staging window per parity
 * (double-buffered so the next chunk's copy overlaps the current step) and an
 * [audio history | AM] window.
 *
 * chunkSamples must be a multiple of rfDecimation * audioDecimation and at least
 * rfTapCount + audioTapCount * rfDecimation (so the first step yields audio).
 * Taps are host memory (copied). hostSlots > 0 adds a ring of pinned (hipHostMalloc) input /
 * output slots for gsdrAmChainStepHost; its H2D copies run on a second stream and overlap the
 * previous step's compute.
 */
typedef struct gsdrAmChainImpl* gsdrAmChain;

typedef struct {
  const float* rfTaps;
  size_t rfTapCount;
  size_t rfDecimation;
  const float* audioTaps;
  size_t audioTapCount;
  size_t audioDecimation;
  size_t chunkSamples;
  size_t hostSlots;
} gsdrAmChainConfig;

GSDR_API hipError_t gsdrAmChainCreate(const gsdrAmChainConfig* config, int32_t device, gsdrAmChain* chainOut);
GSDR_API void gsdrAmChainDestroy(gsdrAmChain chain);
/* Stream every step is enqueued on (non-blocking, created with the chain). */
GSDR_API hipStream_t gsdrAmChainStream(gsdrAmChain chain);
/* Audio samples the NEXT step will produce. */
GSDR_API size_t gsdrAmChainNextOutputCount(gsdrAmChain chain);
/* One step from device memory: chunkSamples IQ pairs at inputIq (copied into the staging window),
 * audio written to `output` (device, gsdrAmChainNextOutputCount floats). Asynchronous. */
GSDR_API hipError_t gsdrAmChainStep(gsdrAmChain chain, const int8_t* inputIq, float* output, size_t* outputCount);
/* nChunks consecutive chunk steps in ONE launch: the chunks are contiguous at inputIq (device), and
 * the audio of all of them is written contiguously at `output` (gsdrAmChainChunksOutputCount
 * floats), exactly as nChunks gsdrAmChainStep calls would produce. Chunk 0 is copied into the
 * staging window behind the carried history; chunks 1.. are read IN PLACE (their RF history is the
 * previous chunk's tail), so the input must stay valid and unmodified until the launch completes
 * (e.g. until the chain stream is synchronised). The whole sequence is one graph; graphs are cached
 * for the last (inputIq, nChunks, output), one per starting state (either staging parity, or the
 * stream's first step), so an odd nChunks does not recapture on every call. */
GSDR_API size_t gsdrAmChainChunksOutputCount(gsdrAmChain chain, size_t nChunks);
GSDR_API hipError_t gsdrAmChainStepChunks(gsdrAmChain chain, const int8_t* inputIq, size_t nChunks, float* output,
                                          size_t* outputCount);
/* Pinned ring. Fill input slot k (chunkSamples IQ pairs), call StepHost(k); after WaitSlot(k) the
 * output slot k holds *outputCount audio samples. A slot may be refilled after its WaitSlot. */
GSDR_API int8_t* gsdrAmChainHostInputSlot(gsdrAmChain chain, size_t slot);
GSDR_API const float* gsdrAmChainHostOutputSlot(gsdrAmChain chain, size_t slot);
GSDR_API hipError_t gsdrAmChainStepHost(gsdrAmChain chain, size_t slot, size_t* outputCount);
GSDR_API hipError_t gsdrAmChainWaitSlot(gsdrAmChain chain, size_t slot);
/* Resident stream: nChunks consecutive chunks at `inputIq` (device), processed as ONE captured
 * graph of three launches (RF FIR + AM over all nChunks * chunkSamples samples, the audio FIR over
 * the whole AM segment, the audio history carry), audio written to `output` (device). After the
 * first step the chain's RF history is read in place: the rfTapCount - 1 (+ < rfDecimation)
 * samples in front of inputIq must be the stream's preceding samples, as they are in a contiguous
 * stream buffer. The graph is cached for the last (inputIq, nChunks, output) and replayed. Output
 * count: gsdrAmChainResidentOutputCount. Do not interleave with gsdrAmChainStep/StepHost on the
 * same stream position (those keep the RF history in the staging window instead). */
GSDR_API size_t gsdrAmChainResidentOutputCount(gsdrAmChain chain, size_t nChunks);
GSDR_API hipError_t gsdrAmChainStepResident(gsdrAmChain chain, const int8_t* inputIq, size_t nChunks, float* output,
                                            size_t* outputCount);
/* Every step entry first checks for a wave-specialised abort counted on the device (a host peek;
 * when set, the chain's streams are synchronised and the count taken): it fails the call with
 * hipErrorLaunchTimeOut. Cached graphs bake in the kernel policy, the FFT guard ratio and the WS
 * spin limit of their capture; a step after any of them changed recaptures. */
/* Graphs the chain has instantiated so far (three at creation, plus every StepChunks /
 * StepResident capture): diagnostics, e.g. to check that steady-state calls replay. */
GSDR_API size_t gsdrAmChainGraphCaptures(gsdrAmChain chain);
/* Forget all history: the next step is a first step again. */
GSDR_API hipError_t gsdrAmChainReset(gsdrAmChain chain);

/*
 * Time-sharded stream (the native form of gpusdr/shard.py's HaloRing, for C /
 * C++ callers): one executor per rank. In step s, rank g of G owns stream samples
 * [(s G + g) L, (s G + g + 1) L) and filters [halo | segment], the halo being the T - 1 samples in
 * front of the segment: rank g - 1's tail of the same step, or, for rank 0, rank G - 1's tail of the
 * previous step (zeros before the first step unless primed through gsdrShardStreamHalo). Outputs
 * L / D per step, the stream's outputs from index (s G + g) L / D on, exactly as one FIR over the
 * whole stream fed T - 1 zeros first (Fir.cpp:178-186 count rule). At G = 1 the halo is the rank's
 * own previous tail (one launch over [halo | segment] plus a T - 1 sample copy).
 *
 * A step enqueues on `stream`: the bulk launch (outputs whose windows lie in the segment) while the
 * caller's exchange moves the tail to rank g + 1 and the halo from rank g - 1 on the executor's
 * second stream, then the head launch (outputs that read the halo; rank 0 uses the halo received
 * one step earlier and never waits). The exchange is the caller's transport:
 *   exchange(user, sendTail, recvHalo, bytes, nextRank, prevRank, xstream) enqueues on (or performs
 *   before returning, ordered after earlier work on) `xstream` the send of `bytes` device bytes at
 *   sendTail to nextRank and the receive of `bytes` from prevRank into recvHalo (device).
 * gsdrShardExchangeRccl is such a hook over an RCCL communicator (user = the ncclComm_t; librccl is
 * loaded on first use, one GPU per rank).
 * With world = 1 and an exchange hook the executor runs the ring protocol on a ring of one (bulk beside
 * the exchange, head from the halo received one step earlier): the rank sends its tail to itself, as
 * rank 0 of a G-rank ring receives rank G - 1's (an RCCL self send / receive exercises the whole
 * protocol on one GPU). Without a hook, world = 1 is one launch plus the history copy.
 *
 * input: int8Iq != 0 -> interleaved int8 IQ (2 bytes per sample), else cf32; output: am != 0 -> the
 * AM envelope (float), else cf32 FIR outputs. L must be a multiple of D and >= T - 1; taps are host
 * memory (copied).
 */
typedef struct gsdrShardStreamImpl* gsdrShardStream;
typedef hipError_t (*gsdrHaloExchangeFn)(void* user, const void* sendTail, void* recvHalo, size_t bytes,
                                         int32_t nextRank, int32_t prevRank, hipStream_t xstream);
GSDR_API hipError_t gsdrShardStreamCreate(int32_t rank, int32_t world, int32_t int8Iq, int32_t am,
                                          const float* taps, size_t tapCount, size_t decimation, size_t segmentSamples,
                                          gsdrHaloExchangeFn exchange, void* user, int32_t device,
                                          gsdrShardStream* streamOut);
GSDR_API void gsdrShardStreamDestroy(gsdrShardStream s);
/* Device address of the segment (segmentSamples samples) the next step filters: write the next
 * segment there (ordered before the step on its stream). */
GSDR_API void* gsdrShardStreamSegment(gsdrShardStream s);
/* Device address of the halo (tapCount - 1 samples in front of the segment), e.g. to prime the
 * first step with the stream's preceding samples. */
GSDR_API void* gsdrShardStreamHalo(gsdrShardStream s);
/* Outputs per step: segmentSamples / decimation. */
GSDR_API size_t gsdrShardStreamOutputCount(gsdrShardStream s);
/* One step; `output` (device) receives gsdrShardStreamOutputCount outputs. Asynchronous on
 * `stream`; the next segment may be written on `stream` after it returns. */
GSDR_API hipError_t gsdrShardStreamStep(gsdrShardStream s, void* output, hipStream_t stream);
GSDR_API hipError_t gsdrShardExchangeRccl(void* ncclComm, const void* sendTail, void* recvHalo, size_t bytes,
                                          int32_t nextRank, int32_t prevRank, hipStream_t xstream);
/* RCCL plumbing for native callers of gsdrShardExchangeRccl (librccl loaded on first use):
 * GetUniqueId fills the 128-byte ncclUniqueId rank 0 hands to every rank; CommCreate makes this rank's
 * communicator on `device` (ncclCommInitRank); CommDestroy frees it. When an RCCL call fails, these and
 * gsdrShardExchangeRccl return hipErrorUnknown (hipErrorSharedObjectInitFailed: librccl missing) and
 * gsdrShardRcclLastResult returns the calling thread's last ncclResult_t (0 = success) and, through
 * `message` if non-null, RCCL's text for it; the failure is also logged through gslog. */
GSDR_API hipError_t gsdrShardRcclGetUniqueId(void* uniqueId128);
GSDR_API hipError_t gsdrShardRcclCommCreate(int32_t nranks, const void* uniqueId128, int32_t rank, int32_t device,
                                            void** ncclCommOut);
GSDR_API hipError_t gsdrShardRcclCommDestroy(void* ncclComm);
GSDR_API int32_t gsdrShardRcclLastResult(const char** message);

#ifdef __cplusplus
}
#endif

#endif /* GSDR_GSDR_AMD_H */
