/*
 * Precondition and HIP-error helpers (MI355X build of the reference's GSErrors.h:28-215 and
 * CudaErrors.h:25-198). hipErrorToStatus keeps the reference's cudaErrorToStatus mapping
 * (CudaErrors.h:25-44); the SAFE_HIP_* macros log the failing call and return a Status /
 * error Result, exactly where the reference's SAFE_CUDA_* macros did.
 */
#ifndef GPUSDRPIPELINE_ABI_ERRORS_H
#define GPUSDRPIPELINE_ABI_ERRORS_H

#include <gpusdrpipeline/abi/core.h>
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <iostream>
#include <sstream>

#define SSTREAM(x) dynamic_cast<std::ostringstream&&>(std::ostringstream() << x).str()

#define GS_FAIL(x)                                                              \
  do {                                                                          \
    std::cerr << SSTREAM(x) << " at " << __FILE__ << ':' << __LINE__ << std::endl; \
    abort();                                                                    \
  } while (false)

#define GS_DETAIL_REQUIRE(cond__, onFalse__)                                                 \
  do {                                                                                       \
    if (!(cond__)) {                                                                         \
      gsloge("Expression must be true [%s] - at %s:%d", #cond__, __FILE__, __LINE__);        \
      onFalse__;                                                                             \
    }                                                                                        \
  } while (false)

#define GS_REQUIRE_OR_RET_STATUS(cond__, msg__) \
  GS_DETAIL_REQUIRE(cond__, { gsloge("%s", msg__); return Status_InvalidArgument; })
#define GS_REQUIRE_OR_RET_STATUS_FMT(cond__, fmt__, ...) \
  GS_DETAIL_REQUIRE(cond__, { gsloge(fmt__, __VA_ARGS__); return Status_InvalidArgument; })
#define GS_REQUIRE_OR_RET_RESULT(cond__, msg__) \
  GS_DETAIL_REQUIRE(cond__, { gsloge("%s", msg__); return ERR_RESULT(Status_InvalidArgument); })
#define GS_REQUIRE_OR_RET_RESULT_FMT(cond__, fmt__, ...) \
  GS_DETAIL_REQUIRE(cond__, { gsloge(fmt__, __VA_ARGS__); return ERR_RESULT(Status_InvalidArgument); })
#define GS_REQUIRE_OR_RET(cond__, msg__, ret__) GS_DETAIL_REQUIRE(cond__, { gsloge("%s", msg__); return ret__; })
#define GS_REQUIRE_OR_RET_FMT(cond__, ret__, fmt__, ...) \
  GS_DETAIL_REQUIRE(cond__, { gsloge(fmt__, __VA_ARGS__); return ret__; })
#define GS_REQUIRE_OR_ABORT(cond__, msg__) GS_DETAIL_REQUIRE(cond__, { gsloge("%s", msg__); abort(); })
#define GS_REQUIRE_OR_THROW(cond__, msg__) \
  GS_DETAIL_REQUIRE(cond__, { gsloge("%s", msg__); throw std::runtime_error("Failed assertion"); })
#define GS_REQUIRE_OR_THROW_FMT(cond__, fmt__, ...) \
  GS_DETAIL_REQUIRE(cond__, { gsloge(fmt__, __VA_ARGS__); throw std::runtime_error("Failed assertion"); })

inline Status hipErrorToStatus(hipError_t e) noexcept {
  switch (e) {
    case hipSuccess: return Status_Success;
    case hipErrorInvalidValue: return Status_InvalidArgument;
    case hipErrorIllegalAddress: return Status_OutOfRange;
    case hipErrorIllegalState: return Status_InvalidState;
    case hipErrorOutOfMemory: return Status_OutOfMemory;
    case hipErrorInvalidDevice:
    case hipErrorFileNotFound:
    case hipErrorSharedObjectSymbolNotFound: return Status_NotFound;
    default: return Status_RuntimeError;
  }
}

#define GS_DETAIL_HIP_CHECK(call__, onErr__)                                                              \
  do {                                                                                                    \
    const hipError_t hipErr__ = (call__);                                                                 \
    if (hipErr__ != hipSuccess) {                                                                         \
      gsloge("HIP error %s (%d) in [%s] at %s:%d", hipGetErrorName(hipErr__), (int)hipErr__, #call__,      \
             __FILE__, __LINE__);                                                                         \
      onErr__;                                                                                            \
    }                                                                                                     \
  } while (false)

#define SAFE_HIP_OR_RET_STATUS(call__) GS_DETAIL_HIP_CHECK(call__, return hipErrorToStatus(hipErr__))
#define SAFE_HIP_OR_RET_RESULT(call__) GS_DETAIL_HIP_CHECK(call__, return ERR_RESULT(hipErrorToStatus(hipErr__)))
#define SAFE_HIP_OR_RET(call__, ret__) GS_DETAIL_HIP_CHECK(call__, return ret__)
#define SAFE_HIP_WARN_ONLY(call__) GS_DETAIL_HIP_CHECK(call__, (void)0)
#define SAFE_HIP_OR_THROW(call__) \
  GS_DETAIL_HIP_CHECK(call__, throw std::runtime_error(hipGetErrorName(hipErr__)))

/* RAII: make `device` current for a scope and restore the caller's device afterwards
 * (reference util/CudaDevicePushPop.h:27-79). */
class HipDevicePushPop final {
 public:
  explicit HipDevicePushPop(int32_t device) noexcept {
    if (hipGetDevice(&mPrev) != hipSuccess) mPrev = -1;
    mStatus = mPrev == device ? hipSuccess : hipSetDevice(device);
  }
  ~HipDevicePushPop() {
    int32_t cur = -1;
    if (mPrev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != mPrev) (void)hipSetDevice(mPrev);
  }
  HipDevicePushPop(const HipDevicePushPop&) = delete;
  HipDevicePushPop& operator=(const HipDevicePushPop&) = delete;
  hipError_t status() const noexcept { return mStatus; }

 private:
  int32_t mPrev = -1;
  hipError_t mStatus = hipSuccess;
};

#define HIP_DEV_PUSH_POP_OR_RET_STATUS(device__)   \
  HipDevicePushPop devPushPop__(device__);         \
  SAFE_HIP_OR_RET_STATUS(devPushPop__.status())
#define HIP_DEV_PUSH_POP_OR_RET_RESULT(device__)   \
  HipDevicePushPop devPushPop__(device__);         \
  SAFE_HIP_OR_RET_RESULT(devPushPop__.status())

#endif  // GPUSDRPIPELINE_ABI_ERRORS_H
