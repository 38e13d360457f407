#include "queues.h"

#include <mutex>
#include <string>
#include <unordered_map>

#include "json.h"

namespace gsdr_rt {

Result<ICudaCommandQueue> HipCommandQueue::create(int32_t device) noexcept {
  HIP_DEV_PUSH_POP_OR_RET_RESULT(device);
  hipStream_t stream = nullptr;
  SAFE_HIP_OR_RET_RESULT(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  auto* q = new (std::nothrow) HipCommandQueue(device, stream);
  if (q == nullptr) {
    (void)hipStreamDestroy(stream);
    return ERR_RESULT(Status_OutOfMemory);
  }
  return makeRefResultNonNull<ICudaCommandQueue>(q);
}

HipCommandQueue::~HipCommandQueue() {
  HipDevicePushPop push(mDevice);
  (void)hipStreamSynchronize(mStream);
  (void)hipStreamDestroy(mStream);
}

namespace {
std::recursive_mutex gQueueLock;
std::unordered_map<std::string, Ref<ICudaCommandQueue>>& namedQueues() {
  static auto* m = new std::unordered_map<std::string, Ref<ICudaCommandQueue>>();  // never destroyed
  return *m;
}
}  // namespace

Status CommandQueueFactory::create(const char* queueId, const char* parameterJson) noexcept {
  try {
    GS_REQUIRE_OR_RET_STATUS(queueId != nullptr, "queueId must not be null");
    std::lock_guard<std::recursive_mutex> l(gQueueLock);
    Json params;
    std::string err;
    if (!Json::parse(parameterJson, params, err) || !params.isObject()) {
      gsloge("Cannot parse command queue parameters [%s]: %s", parameterJson ? parameterJson : "(null)", err.c_str());
      return Status_ParseError;
    }
    const Json* type = params.get("queueType");
    GS_REQUIRE_OR_RET_STATUS(type != nullptr && type->isString(), "queueType (string) is required");
    if (type->string() != "cuda" && type->string() != "hip") {
      gsloge("Unknown queueType [%s]", type->string().c_str());
      return Status_NotFound;
    }
    if (exists(queueId)) return Status_Success;
    int32_t device = 0;
    if (const Json* d = params.get("cudaDevice")) device = (int32_t)d->number();
    Ref<ICudaCommandQueue> q;
    UNWRAP_OR_FWD_STATUS(q, mHipQueues->create(device));
    namedQueues().emplace(queueId, q);
    return Status_Success;
  }
  IF_CATCH_RETURN_STATUS;
}

bool CommandQueueFactory::exists(const char* queueId) noexcept {
  try {
    std::lock_guard<std::recursive_mutex> l(gQueueLock);
    return queueId != nullptr && namedQueues().count(queueId) != 0;
  } catch (...) {
    return false;
  }
}

Result<ICudaCommandQueue> CommandQueueFactory::getCudaCommandQueue(const char* queueId) noexcept {
  try {
    std::lock_guard<std::recursive_mutex> l(gQueueLock);
    if (queueId == nullptr) return ERR_RESULT(Status_InvalidArgument);
    auto it = namedQueues().find(queueId);
    if (it == namedQueues().end()) return ERR_RESULT(Status_NotFound);
    return makeRefResultNonNull<ICudaCommandQueue>(it->second.get().get());
  }
  IF_CATCH_RETURN_RESULT;
}

}  // namespace gsdr_rt

GS_EXPORT Result<int32_t> gsGetCurrentCudaDevice() noexcept {
  int32_t device = -1;
  SAFE_HIP_OR_RET_RESULT(hipGetDevice(&device));
  return makeValResult(device);
}
