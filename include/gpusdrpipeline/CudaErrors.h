#pragma once
/*
 * Reference include path (include/gpusdrpipeline/CudaErrors.h) for drop-in callers: the
 * reference's names forward to the HIP equivalents of gpusdrpipeline/abi/errors.h.
 *   cudaErrorToStatus        -> hipErrorToStatus (same mapping, CudaErrors.h:25-44)
 *   SAFE_CUDA_*              -> SAFE_HIP_* (log the failing call, return / throw)
 *   CHECK_CUDA_*(message)    -> check hipGetLastError() after a kernel launch
 */
#include <gpusdrpipeline/abi/errors.h>

inline Status cudaErrorToStatus(hipError_t e) noexcept { return hipErrorToStatus(e); }

#define SAFE_CUDA_OR_RET(cmd__, ret__) SAFE_HIP_OR_RET(cmd__, ret__)
#define SAFE_CUDA_OR_RET_STATUS(cmd__) SAFE_HIP_OR_RET_STATUS(cmd__)
#define SAFE_CUDA_OR_RET_RESULT(cmd__) SAFE_HIP_OR_RET_RESULT(cmd__)
#define SAFE_CUDA_OR_THROW(cmd__) SAFE_HIP_OR_THROW(cmd__)
#define SAFE_CUDA_WARN_ONLY(cmd__) SAFE_HIP_WARN_ONLY(cmd__)

#define GS_DETAIL_LAST_HIP_ERROR(msg__, onErr__)                                                 \
  do {                                                                                           \
    const hipError_t lastErr__ = hipGetLastError();                                             \
    if (lastErr__ != hipSuccess) {                                                              \
      gsloge("%s: HIP error %s (%d)", (msg__), hipGetErrorName(lastErr__), (int)lastErr__);      \
      onErr__;                                                                                   \
    }                                                                                            \
  } while (false)
#define CHECK_CUDA_OR_RET(msg__, ret__) GS_DETAIL_LAST_HIP_ERROR(msg__, return ret__)
#define CHECK_CUDA_OR_RET_STATUS(msg__) GS_DETAIL_LAST_HIP_ERROR(msg__, return hipErrorToStatus(lastErr__))
#define CHECK_CUDA_OR_RET_RESULT(msg__) \
  GS_DETAIL_LAST_HIP_ERROR(msg__, return ERR_RESULT(hipErrorToStatus(lastErr__)))
#define CHECK_CUDA_OR_THROW(msg__) \
  GS_DETAIL_LAST_HIP_ERROR(msg__, throw std::runtime_error(hipGetErrorName(lastErr__)))
