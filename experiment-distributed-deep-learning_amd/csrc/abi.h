// abi.h — helpers shared by the two C-ABI translation units (c_api.cpp: the deployment surface;
// c_api_testing.cpp: the testing surface).
#pragma once

#include <string>
#include <vector>

#include "common.h"
#include "engine.h"

namespace ddl {
namespace abi {

template <typename F>
inline int guarded(F &&f) {
    try {
        f();
        return DDL_STATUS_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        DDL_LOG(1, "error " << e.status << ": " << e.msg);
        return e.status;
    } catch (const std::exception &e) {
        set_error(e.what());
        return DDL_STATUS_ERROR_UNKNOWN;
    } catch (...) {
        set_error("unknown error");
        return DDL_STATUS_ERROR_UNKNOWN;
    }
}

inline hipStream_t as_stream(void *s) { return static_cast<hipStream_t>(s); }

inline int current_device() {
    int d = 0;
    DDL_HIP(hipGetDevice(&d));
    return d;
}

inline std::vector<std::string> split_endpoints(const char *endpoints) {
    std::vector<std::string> eps;
    std::string s(endpoints);
    size_t pos = 0;
    while (pos <= s.size()) {
        size_t sc = s.find(';', pos);
        if (sc == std::string::npos) sc = s.size();
        if (sc > pos) eps.push_back(s.substr(pos, sc - pos));
        pos = sc + 1;
    }
    return eps;
}

// A tuning table (TuneResult) into the C-ABI's arrays: per candidate {algo, rings, slice_bytes,
// max_slices} and its agreed milliseconds (ddl_tune_result, ddl_local_tune, ddl_rccl_loopback_tune).
inline void export_tune(const TuneResult &r, int *chosen, int *count, long long *configs, float *ms, int max_candidates) {
    DDL_REQUIRE(chosen && count, DDL_STATUS_INVALID_ARGUMENT, "null output");
    *chosen = r.chosen;
    *count = (int)r.candidates.size();
    for (int i = 0; i < *count && i < max_candidates; ++i) {
        const RingConfig &c = r.candidates[i];
        if (configs) {
            configs[4 * i + 0] = c.algo;
            configs[4 * i + 1] = c.rings;
            configs[4 * i + 2] = (long long)c.slice_bytes;
            configs[4 * i + 3] = c.max_slices;
        }
        if (ms) ms[i] = r.ms[i];
    }
}

}  // namespace abi
}  // namespace ddl
