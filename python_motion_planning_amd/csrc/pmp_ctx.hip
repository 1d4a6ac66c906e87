// Context, error channel and grow-only scratch arena of libpmp_hip.so.
#include "pmp_internal.h"

int pmp_set_err(pmp_ctx* ctx, int code, const std::string& msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

void* pmp_scratch(pmp_ctx* ctx, int slot, size_t bytes)
{
    if (bytes == 0) bytes = 16;
    if (ctx->cap[slot] >= bytes) return ctx->buf[slot];
    if (ctx->buf[slot]) {
        (void)hipDeviceSynchronize();  // the old buffer may still be in use by queued work
        (void)hipFree(ctx->buf[slot]);
        ctx->buf[slot] = nullptr;
        ctx->cap[slot] = 0;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        pmp_set_err(ctx, PMP_ENOMEM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
        return nullptr;
    }
    ctx->buf[slot] = p;
    ctx->cap[slot] = bytes;
    return p;
}

extern "C" {

pmp_ctx* pmp_create(int device)
{
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    pmp_ctx* c = new pmp_ctx();
    c->device = device;
    return c;
}

void pmp_destroy(pmp_ctx* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (int i = 0; i < SCR_NSLOTS; i++)
        if (ctx->buf[i]) (void)hipFree(ctx->buf[i]);
    delete ctx;
}

const char* pmp_last_error(pmp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

const char* pmp_version(void) { return "pmp-hip 0.1 gfx950"; }

int pmp_set_timing(pmp_ctx* ctx, uint64_t* span)
{
    if (!ctx) return PMP_EINVAL;
    ctx->span = reinterpret_cast<unsigned long long*>(span);
    return PMP_OK;
}

int pmp_set_stats(pmp_ctx* ctx, int64_t* stats)
{
    if (!ctx) return PMP_EINVAL;
    ctx->stats = reinterpret_cast<unsigned long long*>(stats);
    return PMP_OK;
}

int pmp_wall_clock_khz(pmp_ctx* ctx, int* khz)
{
    if (!ctx || !khz) return PMP_EINVAL;
    PMP_HIP_CHECK(ctx, hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, ctx->device));
    return PMP_OK;
}

int pmp_astar2d_set_schedule(pmp_ctx* ctx, int longest_first)
{
    if (!ctx) return PMP_EINVAL;
    ctx->astar_lpt = longest_first ? 1 : 0;
    return PMP_OK;
}

int pmp_astar2d_set_priority(pmp_ctx* ctx, int n_high)
{
    if (!ctx || n_high < 0) return PMP_EINVAL;
    ctx->astar_prio_n = n_high;
    return PMP_OK;
}

int pmp_set_resident_per_cu(pmp_ctx* ctx, int per_cu)
{
    if (!ctx) return PMP_EINVAL;
    if (per_cu < 0 || per_cu > 32) return pmp_set_err(ctx, PMP_EINVAL, "pmp_set_resident_per_cu: per_cu must be in [0, 32]");
    ctx->resident_per_cu = per_cu;
    return PMP_OK;
}

int pmp_dstar_set_first_cap(pmp_ctx* ctx, int entries)
{
    if (!ctx) return PMP_EINVAL;
    if (entries < 0) return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar_set_first_cap: entries must be >= 0");
    ctx->dstar_first_cap = entries;
    return PMP_OK;
}

int pmp_set_workers_per_cu(pmp_ctx* ctx, int per_cu)
{
    if (!ctx) return PMP_EINVAL;
    if (per_cu < 0 || per_cu > 32) return pmp_set_err(ctx, PMP_EINVAL, "pmp_set_workers_per_cu: per_cu must be in [0, 32]");
    ctx->workers_per_cu = per_cu;
    return PMP_OK;
}

}  // extern "C"
