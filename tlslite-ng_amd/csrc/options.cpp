// options.cpp -- process-wide kernel-selection options (options.h).
#include "options.h"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace tg {
namespace {

struct OptName {
    const char* name;   // tg_set_option name
    const char* env;    // environment variable read once
};

constexpr OptName kNames[kOptCount] = {
    {"gcm_variant", "TLSGPU_GCM_VARIANT"},
    {"gcm_table_variant", "TLSGPU_GCM_TABLE_VARIANT"},
    {"chacha_variant", "TLSGPU_CHACHA_VARIANT"},
    {"ccm_variant", "TLSGPU_CCM_VARIANT"},
    {"waves_per_record", "TLSGPU_WAVES_PER_RECORD"},
    {"no_plan", "TLSGPU_NO_PLAN"},
    {"stage_copy", "TLSGPU_STAGE_COPY"},
    {"hy_t", "TLSGPU_HY_T"},
    {"hy_prio", "TLSGPU_HY_PRIO"},
    {"kt_split", "TLSGPU_KT_SPLIT"},
    {"kt_lpr", "TLSGPU_KT_LPR"},
    {"hy_threads", "TLSGPU_HY_THREADS"},
    {"kt_hybrid", "TLSGPU_KT_HYBRID"},
    {"kt_t", "TLSGPU_KT_T"},
    {"kt_overlap", "TLSGPU_KT_OVERLAP"},
    {"ccm_hy_t", "TLSGPU_CCM_HY_T"},
};

std::atomic<int> g_val[kOptCount];
std::once_flag g_once;

void init_from_env() {
    for (int i = 0; i < kOptCount; ++i) {
        const char* e = getenv(kNames[i].env);
        g_val[i].store(e ? atoi(e) : 0, std::memory_order_relaxed);
    }
}

}  // namespace

int opt(Opt o) {
    std::call_once(g_once, init_from_env);
    return g_val[o].load(std::memory_order_relaxed);
}

void opt_set(Opt o, int value) {
    std::call_once(g_once, init_from_env);
    g_val[o].store(value, std::memory_order_relaxed);
}

int opt_index(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < kOptCount; ++i)
        if (!strcmp(name, kNames[i].name)) return i;
    return -1;
}

}  // namespace tg
