// Thread-local error reporting for the C ABI (llm_last_error).
#include <string>

#include "common.hpp"

namespace llm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int status, const std::string& msg) {
  g_last_error = msg;
  return status;
}

}  // namespace llm

extern "C" const char* llm_last_error(void) { return llm::g_last_error.c_str(); }

extern "C" int llm_abi_version(void) { return 3; }
