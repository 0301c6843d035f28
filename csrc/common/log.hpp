// Logging: LOG(level) << ... ; level from env PCCL_LOG_LEVEL (TRACE, DEBUG, INFO, WARN, ERR, FATAL, NONE).
// Default ERR, like the reference (log/src/pccl_log.cpp:28-56). Unlike the reference, FATAL/BUG never exit the
// process from library code: they only log.
#pragma once

#include <sstream>
#include <string>

namespace pccl {

enum class LogLevel : int { TRACE = 0, DEBUG = 1, INFO = 2, WARN = 3, ERR = 4, FATAL = 5, BUG = 6, NONE = 7 };

LogLevel current_log_level();
void set_log_level(LogLevel level);

class LogLine {
public:
    explicit LogLine(LogLevel level, const char *file, int line);
    ~LogLine();
    template<typename T>
    LogLine &operator<<(const T &v) {
        stream_ << v;
        return *this;
    }

private:
    LogLevel level_;
    std::ostringstream stream_;
};

} // namespace pccl

#define PCCL_LOG_ENABLED(lvl) (static_cast<int>(::pccl::LogLevel::lvl) >= static_cast<int>(::pccl::current_log_level()))
#define LOG(lvl)                                                                                                       \
    if (!PCCL_LOG_ENABLED(lvl)) {                                                                                      \
    } else                                                                                                             \
        ::pccl::LogLine(::pccl::LogLevel::lvl, __FILE__, __LINE__)
