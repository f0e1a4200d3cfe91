// Diagnostic log of the library's slow host-side steps (UPLINK_EC_LOG=1):
// every run-time compilation of an encoder (hiprtc), every load of a
// straight-line decode module, and what process exit waits for -- each with
// its duration -- on stderr, stamped with the milliseconds since the first
// line.  Off by default; read once per process.
#pragma once
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

namespace uplink_ec {

inline bool log_on() {
    static const bool on = [] {
        const char *e = getenv("UPLINK_EC_LOG");
        return e && *e && *e != '0';
    }();
    return on;
}

inline double log_ms() {
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

__attribute__((format(printf, 1, 2))) inline void ec_logf(const char *fmt, ...) {
    if (!log_on()) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    fprintf(stderr, "uplink_ec log [%10.1f ms] %s\n", log_ms(), buf);
}

}  // namespace uplink_ec
