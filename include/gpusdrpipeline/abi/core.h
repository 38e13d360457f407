/*
 * gpusdrpipeline core ABI (MI355X build).
 *
 * Layout- and vtable-compatible restatement of the reference's core interfaces so that code
 * written against kernrj/cuda-sdr's public headers compiles and links against this library:
 *   IRef / ImmutableRef / StealableRef / Ref / RefCt   reference include/gpusdrpipeline/IRef.h:30-301
 *   Status + throwIfError                              Status.h:22-78
 *   RefResult / ValResult (pack 8) + helper macros     Result.h:28-394
 *   logging entry points                               GSLog.h:27-56
 *   export / ref-count macros                          GSDefs.h:23-64
 *   SampleType, Modulation, IMemory                    SampleType.h:20-25, Modulation.h:22-26, IMemory.h:22-40
 *
 * Ownership convention (unchanged): objects are created "floating" with a ref-count of 0, the
 * first Ref/ImmutableRef takes the first reference, and unref() at 0 or 1 destroys. Nothing
 * throws across the boundary: every interface method is noexcept and reports a Status.
 */
#ifndef GPUSDRPIPELINE_ABI_CORE_H
#define GPUSDRPIPELINE_ABI_CORE_H

#include <atomic>
#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <new>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>

#if defined(__clang__)
/* RefResult / ValResult are returned by value from the GS_EXPORT functions (a 16-byte POD
 * {uint32 status; T value} under pack(8)), exactly as in the reference. */
#pragma clang diagnostic ignored "-Wreturn-type-c-linkage"
#endif

/* ---------------------------------------------------------------------------------------------
 * Export and class-shape macros
 * ------------------------------------------------------------------------------------------- */
#if defined(__GNUC__)
#define GS_PUBLIC __attribute__((visibility("default")))
#else
#define GS_PUBLIC
#endif
#define GS_C_LINKAGE extern "C"
#define GS_EXPORT GS_C_LINKAGE GS_PUBLIC

#ifdef __GNUC__
#define GS_FMT_ATTR(FMT_OFFSET, PARAM_OFFSET) __attribute__((format(printf, FMT_OFFSET, PARAM_OFFSET)))
#else
#define GS_FMT_ATTR(FMT_OFFSET, PARAM_OFFSET)
#endif
#define GS_FMT_STR(p) p

/* Abstract interfaces: protected default ctor and virtual dtor. */
#define ABSTRACT_IREF(CLASS_NAME__)  \
 protected:                          \
  CLASS_NAME__() noexcept = default; \
  ~CLASS_NAME__() override = default;

/* Concrete ref-counted classes: ref()/unref() delegate to an embedded RefCt that deletes. */
#define REF_COUNTED_NO_DESTRUCTOR(CLASS_TYPE__)                                \
 public:                                                                       \
  void ref() const noexcept final { mRefCt.ref(); }                            \
  void unref() const noexcept final { mRefCt.unref(); }                        \
                                                                               \
 private:                                                                      \
  static void mSelfDeleter(CLASS_TYPE__* selfPtr) noexcept { delete selfPtr; } \
  RefCt<CLASS_TYPE__> mRefCt { this, mSelfDeleter }

#define REF_COUNTED(REF_CT_CLASS_TYPE__)  \
 private:                                 \
  ~REF_CT_CLASS_TYPE__() final = default; \
  REF_COUNTED_NO_DESTRUCTOR(REF_CT_CLASS_TYPE__)

/* ---------------------------------------------------------------------------------------------
 * Reference counting
 * ------------------------------------------------------------------------------------------- */
class IRef {
 public:
  virtual void ref() const noexcept = 0;
  virtual void unref() const noexcept = 0;

 protected:
  IRef() noexcept = default;
  virtual ~IRef() = default;
};

/* Holds one reference for its whole lifetime; cannot be re-seated. */
template <typename T>
class ImmutableRef final {
 public:
  ImmutableRef() noexcept : mObj(nullptr) {}
  ImmutableRef(T* obj) noexcept : mObj(obj) { acquire(); }
  ImmutableRef(const ImmutableRef<T>& other) noexcept : mObj(other.mObj) { acquire(); }
  ImmutableRef(ImmutableRef<T>&& other) noexcept : mObj(other.mObj) { acquire(); }
  ~ImmutableRef() noexcept {
    if (mObj != nullptr) mObj->unref();
  }
  ImmutableRef& operator=(const ImmutableRef<T>&) = delete;
  ImmutableRef& operator=(ImmutableRef<T>&&) = delete;

  operator T*() const noexcept { return mObj; }
  T* operator->() const noexcept { return mObj; }
  T* get() const noexcept { return mObj; }
  bool operator==(const ImmutableRef<T>& o) const noexcept { return mObj == o.mObj; }
  bool operator!=(const ImmutableRef<T>& o) const noexcept { return mObj != o.mObj; }
  bool operator==(T* o) const noexcept { return mObj == o; }
  bool operator!=(T* o) const noexcept { return mObj != o; }

 private:
  void acquire() noexcept {
    if (mObj != nullptr) mObj->ref();
  }
  T* const mObj;
};

template <typename T>
using ConstRef = const ImmutableRef<T>;

/* Atomically swappable slot that can hand its reference out (steal). */
template <typename T>
class StealableRef final {
 public:
  StealableRef() noexcept : mObj(nullptr) {}
  explicit StealableRef(T* obj) noexcept : mObj(obj) {
    if (obj != nullptr) obj->ref();
  }
  ~StealableRef() {
    if (T* o = steal()) o->unref();
  }
  StealableRef& operator=(T* obj) {
    if (obj != nullptr) obj->ref();
    if (T* old = mObj.exchange(obj)) old->unref();
    return *this;
  }
  T* steal() noexcept { return mObj.exchange(nullptr); }
  operator ImmutableRef<T>() const noexcept { return ImmutableRef<T>(mObj.load()); }
  ImmutableRef<T> operator->() const noexcept { return ImmutableRef<T>(mObj.load()); }
  ImmutableRef<T> get() const noexcept { return ImmutableRef<T>(mObj.load()); }

 private:
  std::atomic<T*> mObj;
};

class IRef;
/* Re-seatable, thread-safe owning reference. */
template <typename T, typename = typename std::enable_if<std::is_base_of<IRef, T>::value>::type>
class Ref final {
 public:
  Ref() noexcept : mObj(nullptr) {}
  Ref(T* obj) noexcept : mObj(nullptr) { reset(obj); }
  Ref(const Ref& o) noexcept : mObj(nullptr) { reset(o.mObj.load()); }
  Ref(Ref&& o) noexcept : mObj(nullptr) {
    reset(o.mObj.load());
    o.reset();
  }
  Ref(const ImmutableRef<T>& o) noexcept : mObj(nullptr) { reset(o.get()); }
  ~Ref() noexcept {
    if (T* o = mObj.load()) o->unref();
  }

  Ref& operator=(T* obj) noexcept {
    reset(obj);
    return *this;
  }
  Ref& operator=(const Ref& o) noexcept {
    if (&o != this) reset(o.mObj.load());
    return *this;
  }
  Ref& operator=(const ImmutableRef<T>& o) noexcept {
    reset(o.get());
    return *this;
  }
  Ref& operator=(Ref&& o) noexcept {
    if (&o != this) {
      reset(o.mObj.load());
      o.reset();
    }
    return *this;
  }

  void reset() noexcept { reset(nullptr); }
  void reset(T* obj) noexcept {
    if (obj != nullptr) obj->ref();  // ref first: obj may already be held here
    T* old = mObj.exchange(obj);
    if (old != nullptr) old->unref();
  }

  operator ImmutableRef<T>() const noexcept { return ImmutableRef<T>(mObj.load()); }
  ImmutableRef<T> operator->() const noexcept { return ImmutableRef<T>(mObj.load()); }
  ImmutableRef<T> get() const noexcept { return ImmutableRef<T>(mObj.load()); }
  bool operator==(const Ref<T>& o) const noexcept { return mObj.load() == o.mObj.load(); }
  bool operator!=(const Ref<T>& o) const noexcept { return mObj.load() != o.mObj.load(); }
  bool operator==(T* o) const noexcept { return mObj.load() == o; }
  bool operator!=(T* o) const noexcept { return mObj.load() != o; }

 private:
  std::atomic<T*> mObj;
};

/* Intrusive counter starting at 0 ("floating"); unref() at 0 or 1 invokes the deleter. */
template <class T>
class RefCt final {
 public:
  RefCt(T* context, void (*onZero)(T* context) noexcept) noexcept : mContext(context), mOnZero(onZero) {}
  RefCt(const RefCt<T>&) = delete;
  RefCt(RefCt<T>&&) = delete;
  RefCt& operator=(const RefCt&) = delete;
  RefCt& operator=(RefCt&&) = delete;
  ~RefCt() = default;

  void ref() const noexcept { mCount.fetch_add(1); }
  void unref() const noexcept {
    size_t prev = mCount.load();
    while (prev != 0 && !mCount.compare_exchange_weak(prev, prev - 1)) {
    }
    if (prev <= 1) mOnZero(mContext);
  }

 private:
  mutable std::atomic_size_t mCount {0};
  T* const mContext;
  void (*const mOnZero)(T* context) noexcept;
};

/* ---------------------------------------------------------------------------------------------
 * Status
 * ------------------------------------------------------------------------------------------- */
using Status = uint32_t;
enum Status_ {
  Status_Success,
  Status_UnknownError,
  Status_OutOfMemory,
  Status_RuntimeError,
  Status_InvalidArgument,
  Status_InvalidState,
  Status_OutOfRange,
  Status_TimedOut,
  Status_NotFound,
  Status_ParseError,
};

/* Application-side helper: turn an error Status into the matching std exception. */
inline void throwIfError(Status status) {
  switch (status) {
    case Status_Success: return;
    case Status_OutOfMemory: throw std::bad_alloc();
    case Status_InvalidArgument: throw std::invalid_argument("Invalid Argument");
    case Status_OutOfRange: throw std::out_of_range("Out of Range");
    case Status_UnknownError: throw std::runtime_error("Unknown Error");
    case Status_RuntimeError: throw std::runtime_error("Error");
    case Status_InvalidState: throw std::runtime_error("Invalid State");
    case Status_TimedOut: throw std::runtime_error("Timed Out");
    case Status_NotFound: throw std::runtime_error("Not Found");
    case Status_ParseError: throw std::runtime_error("Parse Error");
    default: throw std::runtime_error("Error type [" + std::to_string(status) + "]");
  }
}

/* ---------------------------------------------------------------------------------------------
 * Logging (exported C functions; implemented in the library)
 * ------------------------------------------------------------------------------------------- */
using LogLevel = uint32_t;
enum LogLevel_ {
  GSLOG_TRACE,
  GSLOG_DEBUG,
  GSLOG_INFO,
  GSLOG_WARN,
  GSLOG_ERROR,
  GSLOG_FATAL,
};

class ILogger : public virtual IRef {
 public:
  virtual void log(LogLevel level, const char* msgFmt, va_list args) noexcept = 0;

  ABSTRACT_IREF(ILogger);
};

GS_EXPORT [[nodiscard]] const char* gslogLevelName(LogLevel level) noexcept;
GS_EXPORT void gsvlog(LogLevel level, GS_FMT_STR(const char* fmt), va_list args) noexcept;
GS_EXPORT void gslogSetLogger(ILogger* logger) noexcept;
GS_EXPORT void gslogSetVerbosity(LogLevel level) noexcept;
GS_EXPORT GS_FMT_ATTR(1, 2) void gslogt(GS_FMT_STR(const char* fmt), ...) noexcept;
GS_EXPORT GS_FMT_ATTR(1, 2) void gslogd(GS_FMT_STR(const char* fmt), ...) noexcept;
GS_EXPORT GS_FMT_ATTR(1, 2) void gslogi(GS_FMT_STR(const char* fmt), ...) noexcept;
GS_EXPORT GS_FMT_ATTR(1, 2) void gslogw(GS_FMT_STR(const char* fmt), ...) noexcept;
GS_EXPORT GS_FMT_ATTR(1, 2) void gsloge(GS_FMT_STR(const char* fmt), ...) noexcept;
GS_EXPORT [[noreturn]] GS_FMT_ATTR(1, 2) void gslogf(GS_FMT_STR(const char* fmt), ...) noexcept;

/* ---------------------------------------------------------------------------------------------
 * Results: {status, value}, 8-byte packed. For IRef types the value is a (floating or
 * borrowed) pointer; otherwise it is held by value.
 * ------------------------------------------------------------------------------------------- */
template <typename T>
#pragma pack(push, 8)
struct RefResult {
  using ValueType = T*;
  const Status status;
  T* const value;
};
#pragma pack(pop)

template <typename T>
#pragma pack(push, 8)
struct ValResult {
  using ValueType = T;
  Status status;
  T value;
};
#pragma pack(pop)

template <typename T>
using Result = typename std::conditional<std::is_base_of<IRef, T>::value, RefResult<T>, ValResult<T>>::type;

template <typename T>
ImmutableRef<T> unwrap(RefResult<T>* result) {
  ImmutableRef<T> value = result->value;
  result->value = nullptr;
  throwIfError(result->status);
  return value;
}

template <typename T>
ImmutableRef<T> unwrap(RefResult<T>&& result) {
  ImmutableRef<T> value = result.value;
  throwIfError(result.status);
  return value;
}

template <typename T>
T* unwrapRaw(RefResult<T>&& result) {
  if (result.status != Status_Success && result.value != nullptr) result.value->unref();
  throwIfError(result.status);
  return result.value;
}

template <typename T>
T unwrap(ValResult<T>* result) {
  throwIfError(result->status);
  return result->value;
}

template <typename T>
T unwrap(ValResult<T>&& result) {
  throwIfError(result.status);
  return result.value;
}

template <typename Out, typename In>
inline RefResult<Out> ResultCast(const RefResult<In>& r) noexcept {
  return {.status = r.status, .value = r.value};
}
template <typename Out, typename In>
inline RefResult<Out> ResultCast(RefResult<In>&& r) noexcept {
  return {.status = r.status, .value = r.value};
}
template <typename Out, typename In>
inline ValResult<Out> ResultCast(const ValResult<In>& r) noexcept {
  return {.status = r.status, .value = r.value};
}
template <typename Out, typename In>
inline ValResult<Out> ResultCast(ValResult<In>&& r) noexcept {
  return {.status = r.status, .value = std::move(r.value)};
}

template <typename T>
RefResult<T> makeRefResultNonNull(T* obj) noexcept {
  return {.status = obj != nullptr ? Status_Success : Status_OutOfMemory, .value = obj};
}
template <typename T>
RefResult<T> makeRefResultNonNull(const ImmutableRef<T>& obj) noexcept {
  return {.status = obj != nullptr ? Status_Success : Status_OutOfMemory, .value = obj};
}
template <typename T>
Result<T> makeRefResultNullable(T* obj) noexcept {
  return {.status = Status_Success, .value = obj};
}
template <typename T>
Result<T> makeValResult(T value) noexcept {
  return {.status = Status_Success, .value = value};
}
template <typename T>
Result<T> errResult(Status status) {
  return {.status = status, .value = {}};
}

#define ERR_RESULT(errResultStatus__) \
  { .status = errResultStatus__, .value = {} }

#define CAST_RESULT(resultCmd__)                                                  \
  do {                                                                            \
    auto castRes__ = resultCmd__;                                                 \
    return {.status = castRes__.status, .value = std::move(castRes__.value)};     \
  } while (false)

#define GS_DETAIL_LOG_RESULT_ERR(what__) gsloge("Error in result [%s] at %s:%d", what__, __FILE__, __LINE__)
#define GS_DETAIL_LOG_STATUS_ERR(st__) gsloge("Error [%u] at %s:%d", (unsigned)(st__), __FILE__, __LINE__)

#define UNWRAP_OR_FWD_RESULT(assignValueToVar__, unwrapCmd__)     \
  do {                                                            \
    auto res__ = unwrapCmd__;                                     \
    if (res__.status != Status_Success) {                         \
      GS_DETAIL_LOG_RESULT_ERR(#unwrapCmd__);                     \
      return {.status = res__.status, .value = {}};               \
    }                                                             \
    assignValueToVar__ = res__.value;                             \
  } while (false)

#define UNWRAP_MOVE_OR_FWD_RESULT(assignValueToVar__, unwrapCmd__) \
  do {                                                             \
    auto res__ = unwrapCmd__;                                      \
    if (res__.status != Status_Success) {                          \
      GS_DETAIL_LOG_RESULT_ERR(#unwrapCmd__);                      \
      return {.status = res__.status, .value = {}};                \
    }                                                              \
    assignValueToVar__ = std::move(res__.value);                   \
  } while (false)

#define UNWRAP_OR_FWD_STATUS(assignValueToVar__, unwrapCmd__) \
  do {                                                        \
    auto res__ = unwrapCmd__;                                 \
    if (res__.status != Status_Success) {                     \
      GS_DETAIL_LOG_RESULT_ERR(#unwrapCmd__);                 \
      return res__.status;                                    \
    }                                                         \
    assignValueToVar__ = res__.value;                         \
  } while (false)

#define UNWRAP_OR_RETURN(assignValueToVar__, unwrapCmd__, retOnError__) \
  do {                                                                  \
    auto res__ = unwrapCmd__;                                           \
    if (res__.status != Status_Success) {                               \
      GS_DETAIL_LOG_RESULT_ERR(#unwrapCmd__);                           \
      return retOnError__;                                              \
    }                                                                   \
    assignValueToVar__ = res__.value;                                   \
  } while (false)

#define DO_OR_FWD_ERR(unwrapCmd__)                      \
  do {                                                  \
    auto res__ = unwrapCmd__;                           \
    if (res__.status != Status_Success) {               \
      GS_DETAIL_LOG_RESULT_ERR(#unwrapCmd__);           \
      return {.status = res__.status, .value = {}};     \
    }                                                   \
  } while (false)

#define WARN_IF_ERR(cmdReturningStatus__)                 \
  do {                                                    \
    const Status st__ = cmdReturningStatus__;             \
    if (st__ != Status_Success) GS_DETAIL_LOG_STATUS_ERR(st__); \
  } while (false)

#define FWD_IF_ERR(cmdReturningStatus__)    \
  do {                                      \
    const Status st__ = cmdReturningStatus__; \
    if (st__ != Status_Success) {           \
      GS_DETAIL_LOG_STATUS_ERR(st__);       \
      return st__;                          \
    }                                       \
  } while (false)

#define THROW_IF_ERR(cmdReturningStatus__)  \
  do {                                      \
    const Status st__ = cmdReturningStatus__; \
    if (st__ != Status_Success) {           \
      GS_DETAIL_LOG_STATUS_ERR(st__);       \
      throwIfError(st__);                   \
    }                                       \
  } while (false)

#define RET_IF_ERR(cmdReturningStatus__, returnValueOnErr__) \
  do {                                                       \
    const Status st__ = cmdReturningStatus__;                \
    if (st__ != Status_Success) {                            \
      GS_DETAIL_LOG_STATUS_ERR(st__);                        \
      return returnValueOnErr__;                             \
    }                                                        \
  } while (false)

#define FWD_IN_RESULT_IF_ERR(cmdReturningStatus__)  \
  do {                                              \
    const Status st__ = cmdReturningStatus__;       \
    if (st__ != Status_Success) {                   \
      GS_DETAIL_LOG_STATUS_ERR(st__);               \
      return {.status = st__, .value = {}};         \
    }                                               \
  } while (false)

#define NON_NULL_OR_RET(ptr__)                                              \
  do {                                                                      \
    if ((ptr__) == nullptr) {                                               \
      gsloge("%s cannot be null - at %s:%d", #ptr__, __FILE__, __LINE__);   \
      return ERR_RESULT(Status_OutOfMemory);                                \
    }                                                                       \
  } while (false)

#define NON_NULL_PARAM_OR_RET(ptr__)                                        \
  do {                                                                      \
    if ((ptr__) == nullptr) {                                               \
      gsloge("%s cannot be null - at %s:%d", #ptr__, __FILE__, __LINE__);   \
      return ERR_RESULT(Status_InvalidArgument);                            \
    }                                                                       \
  } while (false)

#define GS_DETAIL_CATCH_AS(returnMapped__)                                   \
  catch (const std::bad_alloc&) { returnMapped__(Status_OutOfMemory); }      \
  catch (const std::out_of_range&) { returnMapped__(Status_OutOfRange); }    \
  catch (const std::invalid_argument&) { returnMapped__(Status_InvalidArgument); } \
  catch (const std::runtime_error&) { returnMapped__(Status_RuntimeError); } \
  catch (...) { returnMapped__(Status_UnknownError); }

#define GS_DETAIL_RETURN_STATUS(s__) return s__
#define GS_DETAIL_RETURN_RESULT(s__) return ERR_RESULT(s__)

#define IF_CATCH_RETURN_STATUS GS_DETAIL_CATCH_AS(GS_DETAIL_RETURN_STATUS)
#define IF_CATCH_RETURN_RESULT GS_DETAIL_CATCH_AS(GS_DETAIL_RETURN_RESULT)

#define DO_OR_RET_STATUS(doCmd__) \
  do {                            \
    try {                         \
      doCmd__;                    \
    }                             \
    IF_CATCH_RETURN_STATUS        \
  } while (false)

#define DO_OR_RET_ERR_RESULT(doCmd__) \
  do {                                \
    try {                             \
      doCmd__;                        \
    }                                 \
    IF_CATCH_RETURN_RESULT            \
  } while (false)

template <class T>
GS_FMT_ATTR(2, 3)
inline bool printIfError(Result<T>&& result, GS_FMT_STR(const char* fmt), ...) noexcept {
  if (result.status != Status_Success) {
    va_list args;
    va_start(args, fmt);
    gsvlog(GSLOG_ERROR, fmt, args);
    va_end(args);
  }
  return std::move(result.value);
}

/* ---------------------------------------------------------------------------------------------
 * Sample formats and modulations
 * ------------------------------------------------------------------------------------------- */
using SampleType = uint32_t;
enum SampleType_ {
  SampleType_FloatComplex,  // interleaved {re, im} float32, 8 bytes
  SampleType_Float,         // float32
  SampleType_Int8Complex,   // interleaved int8 I, Q
};

using Modulation = uint32_t;
enum Modulation_ {
  Modulation_Am,
  Modulation_Fm,
};

/* A block of memory (device, pinned host or system) owned through ref-counting. */
class IMemory : public virtual IRef {
 public:
  [[nodiscard]] virtual uint8_t* data() noexcept = 0;
  [[nodiscard]] virtual const uint8_t* data() const noexcept = 0;
  [[nodiscard]] virtual size_t capacity() const noexcept = 0;

  template <typename T = uint8_t>
  [[nodiscard]] T* as() noexcept {
    return reinterpret_cast<T*>(data());
  }
  template <typename T = uint8_t>
  [[nodiscard]] const T* as() const noexcept {
    return reinterpret_cast<const T*>(data());
  }

  ABSTRACT_IREF(IMemory);
};

#endif  // GPUSDRPIPELINE_ABI_CORE_H
