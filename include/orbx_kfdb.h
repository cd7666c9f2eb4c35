/* orbx_kfdb.h — C ABI of the keyframe database (replaces ORB_SLAM2::KeyFrameDatabase,
 * include/KeyFrameDatabase.h:40-66, src/KeyFrameDatabase.cc).
 *
 * The reference keeps an inverted file (word -> list of KeyFrame*, in add order) and, on
 * the KeyFrame objects, the per-query state its two detectors write (mnRelocQuery,
 * mnRelocWords, mRelocScore, mnLoopQuery, mnLoopWords, mLoopScore).  Here the database is
 * resident in HBM: every keyframe's BowVector (word ids ascending, DBoW2 weights), its
 * best-covisibility list (KeyFrame::GetBestCovisibilityKeyFrames(N), as the Map maintains it)
 * and the persistent score state, indexed by slot = the order of add().  A query scans the
 * whole database on the GPU (shared words, L1 score and first shared query word per
 * keyframe), then one workgroup runs the candidate selection of the reference: the
 * 0.8*maxCommonWords filter, the covisibility accumulation, the 0.75*bestAccScore retention
 * and the de-duplicated candidate list in the reference's list order.
 *
 * The caller maps KeyFrame* <-> slot.  Conventions where the reference is undefined:
 *   - mRelocScore starts at 0 (the reference leaves it uninitialised; it is read for
 *     neighbours that share a word with the frame but were not scored by the current query,
 *     i.e. the value the previous relocalisation query left, which the slot state keeps);
 *   - every detect call is a new query id (the reference passes F->mnId / pKF->mnId, unique
 *     per frame / keyframe).
 * Host-pointer entry points copy their inputs and wait (like the reference's calls).
 */
#ifndef ORBX_KFDB_H
#define ORBX_KFDB_H

#include "orbx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orbx_kfdb orbx_kfdb;

typedef struct {
    int32_t covisibles;   /* neighbours kept per keyframe: GetBestCovisibilityKeyFrames(10)
                             at KeyFrameDatabase.cc:162 / :292 (1 .. 64) */
    int32_t device;       /* HIP device ordinal */
} orbx_kfdb_params;

/* KeyFrameDatabase::KeyFrameDatabase (:33-37). */
orbx_status orbx_kfdb_create(const orbx_kfdb_params* params, orbx_kfdb** out);
orbx_status orbx_kfdb_destroy(orbx_kfdb* db);

/* KeyFrameDatabase::add (:40-46): appends a keyframe with BowVector (words[n] strictly
 * ascending, values[n]); *slot = its index (its position in every inverted-file list). */
orbx_status orbx_kfdb_add(orbx_kfdb* db, const uint32_t* words, const double* values, int32_t n,
                          int32_t* slot);
/* KeyFrameDatabase::erase (:48-67): the slot leaves every inverted-file list. */
orbx_status orbx_kfdb_erase(orbx_kfdb* db, int32_t slot);
/* KeyFrameDatabase::clear (:69-73): empties the database (slots restart at 0). */
orbx_status orbx_kfdb_clear(orbx_kfdb* db);
orbx_status orbx_kfdb_size(const orbx_kfdb* db, int32_t* nslots);

/* The slot's KeyFrame::GetBestCovisibilityKeyFrames result (mvpOrderedConnectedKeyFrames,
 * weight-descending; KeyFrame.cc:142-186) as slots; the first `covisibles` are kept.  Call
 * it whenever the Map updates the keyframe's connections (KeyFrame::UpdateConnections). */
orbx_status orbx_kfdb_set_covisibles(orbx_kfdb* db, int32_t slot, const int32_t* neighbours,
                                     int32_t n);

/* KeyFrameDatabase::DetectRelocalizationCandidates (:220-337) for the frame BowVector
 * (qwords[nq] ascending, qvalues[nq]): cand[*ncand] = candidate slots in the reference's
 * order (ORBX_ERR_CAPACITY if more than cap; *ncand holds the count). */
orbx_status orbx_kfdb_detect_relocalization(orbx_kfdb* db, const uint32_t* qwords,
                                            const double* qvalues, int32_t nq, int32_t* cand,
                                            int32_t cap, int32_t* ncand);

/* KeyFrameDatabase::DetectLoopCandidates (:76-208) for a keyframe BowVector: connected[nc]
 * = the slots of pKF->GetConnectedKeyFrames() (excluded from the candidates), min_score the
 * minScore argument. */
orbx_status orbx_kfdb_detect_loop(orbx_kfdb* db, const uint32_t* qwords, const double* qvalues,
                                  int32_t nq, const int32_t* connected, int32_t nc,
                                  float min_score, int32_t* cand, int32_t cap, int32_t* ncand);

/* Per-kernel time of the last detect call (ms): the database scan and the selection. */
orbx_status orbx_kfdb_last_timing(const orbx_kfdb* db, double* scan_ms, double* select_ms);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_KFDB_H */
