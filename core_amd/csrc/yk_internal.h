// Internal helpers shared by the host and device halves of libyk.
#pragma once
#include <string>

namespace yk {
// records the message as yk_last_error() of this thread and returns code
int set_error(int code, const std::string& msg);
}  // namespace yk
