// Shared host-side helpers: status codes, thread-local error text, HIP checks.
#pragma once
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "mpiasyncpools.h"

namespace mpa {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* last_error();

// A status-carrying failure used inside the library; converted to a code at the C ABI.
struct Failure {
  int code;
};

[[noreturn]] void fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace mpa
