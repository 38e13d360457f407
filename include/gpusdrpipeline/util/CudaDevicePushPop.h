#pragma once
/*
 * Reference include path (include/gpusdrpipeline/util/CudaDevicePushPop.h) for drop-in callers:
 * CudaDevicePushPop and the CUDA_DEV_PUSH_POP_* macros forward to HipDevicePushPop
 * (gpusdrpipeline/abi/errors.h), which makes a device current for a scope and restores the
 * caller's device afterwards.
 */
#include <gpusdrpipeline/CudaErrors.h>

using CudaDevicePushPop = HipDevicePushPop;

#define CUDA_DEV_PUSH_POP_OR_RET(device__, ret__) \
  HipDevicePushPop devPushPop__(device__);        \
  SAFE_HIP_OR_RET(devPushPop__.status(), ret__)
#define CUDA_DEV_PUSH_POP_OR_RET_STATUS(device__) HIP_DEV_PUSH_POP_OR_RET_STATUS(device__)
#define CUDA_DEV_PUSH_POP_OR_RET_RESULT(device__) HIP_DEV_PUSH_POP_OR_RET_RESULT(device__)
#define CUDA_DEV_PUSH_POP_OR_THROW(device__) \
  HipDevicePushPop devPushPop__(device__);   \
  SAFE_HIP_OR_THROW(devPushPop__.status())
