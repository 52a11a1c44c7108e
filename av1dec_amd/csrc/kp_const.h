// kp_const.h -- per-launch frame parameters in the constant address space.
//
// Every field a kernel reads from KParams through a constant-address-space object is a
// scalar load that the compiler may hoist anywhere; the same array behind a plain global
// pointer costs hoisted vector loads (~100 VGPRs in k_inter) or, in the filters, reloads
// inside the pixel loops (the pixel stores might alias it).  Each translation unit with
// kernels owns one table (AV1R_KP_TABLE); launch batches rotate over AV1R_KP_SLOTS slots
// of AV1R_MAX_BATCH frames, and a slot is rewritten only after the previous batch that
// used it has finished (one event per slot, waited for on the GPU, not the host).
#pragma once
#include <mutex>

#include "av1r_dev.h"

struct KpSlots {
    std::mutex m;
    int next = 0;
    hipEvent_t ev[AV1R_KP_SLOTS] = {};
    bool used[AV1R_KP_SLOTS] = {};
};

static inline int kp_upload_impl(KpSlots* slots, const void* symbol, int device, const KParams* host, int n,
    hipStream_t s)
{
    if (device < 0 || device >= 64 || n < 1 || n > AV1R_MAX_BATCH) return -1;
    KpSlots& S = slots[device];
    std::lock_guard<std::mutex> lock(S.m);
    const int slot = S.next;
    S.next = (S.next + 1) % AV1R_KP_SLOTS;
    if (!S.ev[slot] && hipEventCreateWithFlags(&S.ev[slot], hipEventDisableTiming) != hipSuccess) return -1;
    if (S.used[slot] && hipStreamWaitEvent(s, S.ev[slot], 0) != hipSuccess) return -1;
    void* base = nullptr;
    if (hipGetSymbolAddress(&base, symbol) != hipSuccess) return -1;
    uint8_t* dst = static_cast<uint8_t*>(base) + (size_t)slot * AV1R_MAX_BATCH * sizeof(KParams);
    if (hipMemcpyAsync(dst, host, sizeof(KParams) * n, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
    return slot;
}

static inline int kp_release_impl(KpSlots* slots, int device, int slot, hipStream_t s)
{
    KpSlots& S = slots[device];
    std::lock_guard<std::mutex> lock(S.m);
    S.used[slot] = true;
    return hipEventRecord(S.ev[slot], s) == hipSuccess ? 0 : -1;
}

// Defines the table NAME plus host functions UPLOAD (claim a slot, copy n frames' pinned
// KParams into it on stream s; returns the slot or -1) and RELEASE (the last launch
// reading the slot has been queued on s).
#define AV1R_KP_TABLE(NAME, UPLOAD, RELEASE)                                                 \
    __constant__ KParams NAME[AV1R_KP_SLOTS][AV1R_MAX_BATCH];                                \
    static KpSlots NAME##_slots[64];                                                         \
    int UPLOAD(int device, const KParams* host, int n, hipStream_t s)                        \
    {                                                                                        \
        return kp_upload_impl(NAME##_slots, HIP_SYMBOL(NAME), device, host, n, s);           \
    }                                                                                        \
    int RELEASE(int device, int slot, hipStream_t s) { return kp_release_impl(NAME##_slots, device, slot, s); }
