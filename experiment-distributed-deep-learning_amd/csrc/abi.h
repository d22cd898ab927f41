// abi.h — helpers shared by the two C-ABI translation units (c_api.cpp: the deployment surface;
// c_api_testing.cpp: the testing surface).
#pragma once

#include <string>
#include <vector>

#include "common.h"

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

}  // namespace abi
}  // namespace ddl
