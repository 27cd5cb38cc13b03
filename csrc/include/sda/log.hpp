// Leveled stderr logging (the reference uses slog: cli/src/main.rs:83-88,
// server-cli/src/lib.rs:29-36). Levels follow slog: 1=critical 2=error
// 3=warning 4=info 5=debug 6=trace.
#pragma once

#include <string>

namespace sda {

void set_log_level(int level);
int log_level();
void log_at(int level, const std::string& msg);
inline void log_error(const std::string& m) { log_at(2, m); }
inline void log_warn(const std::string& m) { log_at(3, m); }
inline void log_info(const std::string& m) { log_at(4, m); }
inline void log_debug(const std::string& m) { log_at(5, m); }

}  // namespace sda
