// options.h -- process-wide kernel-selection options of libtlsgpu.
//
// The launchers consult these instead of calling getenv on every launch.
// Each option starts from its TLSGPU_* environment variable, read once per
// process on first use, and tg_set_option (include/tlsgpu.h) changes it at
// run time -- the tests force one kernel after another in a single process
// that way.  0 always means "auto" (the engine's own choice).
#pragma once

namespace tg {

enum Opt {
    kOptGcmVariant = 0,       // TLSGPU_GCM_VARIANT: single-key AES-GCM kernel (aes_gcm.hip)
    kOptGcmTableVariant,      // TLSGPU_GCM_TABLE_VARIANT: key-table AES-GCM kernel
    kOptChachaVariant,        // TLSGPU_CHACHA_VARIANT
    kOptCcmVariant,           // TLSGPU_CCM_VARIANT
    kOptWavesPerRecord,       // TLSGPU_WAVES_PER_RECORD: 1 / 4 / 16, 0 = by batch size
    kOptNoPlan,               // TLSGPU_NO_PLAN: 1 = no length-sorted launch order
    kOptStageCopy,            // TLSGPU_STAGE_COPY: 1 = per-record calls copy through HBM
    kOptHyT,                  // TLSGPU_HY_T: T-table waves of the hybrid kernel (0 = 10 of 16)
    kOptHyPrio,               // TLSGPU_HY_PRIO: 1 = T-table waves at raised priority
    kOptKtSplit,              // TLSGPU_KT_SPLIT: key-table length split in bytes, 0 = auto
    kOptKtLpr,                // TLSGPU_KT_LPR: key-table long records, lanes per record
                              // (8 / 16 / 32 / 64), -1 wave-per-record T-table, 0 auto
    kOptHyThreads,            // TLSGPU_HY_THREADS: hybrid AES-GCM workgroup, 0 = 1024, or 768
    kOptKtHybrid,             // TLSGPU_KT_HYBRID: key-table long records on the T-table +
                              // bitsliced persistent kernel (1) or the bitsliced one (-1), 0 auto
    kOptKtT,                  // TLSGPU_KT_T: T-table waves of that kernel (0 = auto)
    kOptKtOverlap,            // TLSGPU_KT_OVERLAP: key-table lane kernel on a second stream beside
                              // the long records' kernel (0 = auto, on; -1 = one stream)
    kOptCcmHyT,               // TLSGPU_CCM_HY_T: T-table waves of the AES-CCM hybrid kernel
                              // (0 = auto, -1 none)
    kOptCount
};

// The option's current value (environment value on first use, 0 if unset).
int opt(Opt o);
// Name -> option, or -1.
int opt_index(const char* name);
void opt_set(Opt o, int value);

}  // namespace tg
