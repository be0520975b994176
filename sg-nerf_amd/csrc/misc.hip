// misc.hip -- error plumbing and ABI version of libsgn_hip.so.
#include "sgn_common.h"

namespace sgn {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
const char *get_error() { return g_last_error.c_str(); }
}  // namespace sgn

extern "C" {
int sgn_abi_version(void) { return SGN_ABI_VERSION; }
const char *sgn_last_error(void) { return sgn::get_error(); }
}
