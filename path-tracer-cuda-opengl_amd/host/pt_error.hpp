// pt_error.hpp — thread-local last-error string behind pt_last_error().
// Replaces checkCudaErrors' print + cudaDeviceReset + exit(99) (utils/cuda_check.h:8-17):
// the library never exits the process; it returns a status code and records a message.
#pragma once
#include <string>

namespace pt {
inline std::string& lastError() {
    static thread_local std::string msg;
    return msg;
}
inline int fail(int code, const std::string& msg) {
    lastError() = msg;
    return code;
}
}  // namespace pt
