// Cross-stream ordering for a handle whose device scratch (or state) is shared by its launches:
// a launch on another stream than the previous one first waits for that one's work, through an
// event recorded after every launch.  Calls on one stream cost nothing extra beyond the record.
// Used by the LZ4 compressor, the AES cipher and the dedup index (their C-ABI entry points take
// a caller stream; SDFS's flush threads may each bring their own).
#pragma once

#include <hip/hip_runtime.h>

namespace sdfs {

struct StreamOrder {
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;
    bool valid = false;

    hipError_t init() { return hipEventCreateWithFlags(&ev, hipEventDisableTiming); }
    // before the launches on s
    hipError_t acquire(hipStream_t s) const {
        return valid && last != s ? hipStreamWaitEvent(s, ev, 0) : hipSuccess;
    }
    // after the launches on s
    hipError_t release(hipStream_t s) {
        const hipError_t e = hipEventRecord(ev, s);
        if (e == hipSuccess) {
            valid = true;
            last = s;
        }
        return e;
    }
    void destroy() {
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
        valid = false;
    }
};

}  // namespace sdfs
