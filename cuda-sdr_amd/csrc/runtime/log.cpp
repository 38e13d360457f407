// Logging entry points (reference GSLog.h:44-56, src/GSLog.cpp): a pluggable ILogger, stderr
// by default, filtered by a process-wide verbosity (INFO unless GSLOG_LEVEL=trace|debug|...).
#include <gpusdrpipeline/abi/core.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace {

std::mutex gLogLock;
ILogger* gLogger = nullptr;  // holds one reference while installed
std::atomic<LogLevel> gVerbosity{GSLOG_INFO};
std::once_flag gEnvOnce;

void readEnvLevel() {
  const char* v = getenv("GSLOG_LEVEL");
  if (v == nullptr) return;
  static const char* names[] = {"trace", "debug", "info", "warn", "error", "fatal"};
  for (LogLevel i = 0; i < 6; ++i)
    if (strcasecmp(v, names[i]) == 0) gVerbosity = i;
}

}  // namespace

GS_EXPORT const char* gslogLevelName(LogLevel level) noexcept {
  switch (level) {
    case GSLOG_TRACE: return "TRACE";
    case GSLOG_DEBUG: return "DEBUG";
    case GSLOG_INFO: return "INFO";
    case GSLOG_WARN: return "WARN";
    case GSLOG_ERROR: return "ERROR";
    case GSLOG_FATAL: return "FATAL";
    default: return "UNKNOWN";
  }
}

GS_EXPORT void gsvlog(LogLevel level, const char* fmt, va_list args) noexcept {
  std::call_once(gEnvOnce, readEnvLevel);
  if (level < gVerbosity.load()) return;
  std::lock_guard<std::mutex> l(gLogLock);
  if (gLogger != nullptr) {
    gLogger->log(level, fmt, args);
    return;
  }
  fprintf(stderr, "[gpusdr %s] ", gslogLevelName(level));
  vfprintf(stderr, fmt, args);
  const size_t n = strlen(fmt);
  if (n == 0 || fmt[n - 1] != '\n') fputc('\n', stderr);
}

GS_EXPORT void gslogSetLogger(ILogger* logger) noexcept {
  std::lock_guard<std::mutex> l(gLogLock);
  if (logger != nullptr) logger->ref();
  if (gLogger != nullptr) gLogger->unref();
  gLogger = logger;
}

GS_EXPORT void gslogSetVerbosity(LogLevel level) noexcept {
  std::call_once(gEnvOnce, readEnvLevel);
  gVerbosity = level;
}

#define GS_DEFINE_LEVEL_LOG(fn__, level__)     \
  GS_EXPORT void fn__(const char* fmt, ...) noexcept { \
    va_list args;                               \
    va_start(args, fmt);                        \
    gsvlog(level__, fmt, args);                 \
    va_end(args);                               \
  }

GS_DEFINE_LEVEL_LOG(gslogt, GSLOG_TRACE)
GS_DEFINE_LEVEL_LOG(gslogd, GSLOG_DEBUG)
GS_DEFINE_LEVEL_LOG(gslogi, GSLOG_INFO)
GS_DEFINE_LEVEL_LOG(gslogw, GSLOG_WARN)
GS_DEFINE_LEVEL_LOG(gsloge, GSLOG_ERROR)

GS_EXPORT void gslogf(const char* fmt, ...) noexcept {
  va_list args;
  va_start(args, fmt);
  gsvlog(GSLOG_FATAL, fmt, args);
  va_end(args);
  abort();
}
