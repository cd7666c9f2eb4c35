/* orbx_vocab.h — C ABI of the bag-of-words vocabulary (DBoW2 TemplatedVocabulary<FORB>).
 *
 * Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:420-427, src/KeyFrame.cc:59-67) turn
 * a frame's descriptors into the BowVector and the FeatureVector the matchers walk
 * (include/orbx_match.h, orbx_featureset.node_*).  The tree descent runs on the GPU, one lane
 * per descriptor; the sparse vectors are assembled on the host in the reference's order.
 * Replaces Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1123-1256 (transform) and
 * :1338-1417 (loadFromTextFile); BowVector.cpp:34-84; FeatureVector.cpp:31-45;
 * ScoringObject.cpp:23-67 (L1 score).
 */
#ifndef ORBX_VOCAB_H
#define ORBX_VOCAB_H

#include "orbx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orbx_vocabulary orbx_vocabulary;

/* TemplatedVocabulary::loadFromTextFile: first line "k L scoring weighting", then one line
 * per node "parent isLeaf d0 .. d31 weight" (ORBvoc.txt's format).  Blank lines are skipped
 * (the reference turns a trailing one into a node with an unread descriptor). */
orbx_status orbx_vocabulary_load_text(const char* path, int device, orbx_vocabulary** out);
orbx_status orbx_vocabulary_destroy(orbx_vocabulary* v);
orbx_status orbx_vocabulary_info(const orbx_vocabulary* v, int32_t* k, int32_t* L,
                                 int32_t* scoring, int32_t* weighting, int32_t* n_nodes,
                                 int32_t* n_words);

/* transform(features, BowVector&, FeatureVector&, levelsup) on n descriptors (n x 32, host).
 * word/node (n entries each, may be NULL): the leaf word and the level-(L - levelsup) node
 * of every descriptor.  BowVector: bow_n entries (word ascending) in bow_word / bow_value
 * (capacity n).  FeatureVector: fv_n nodes (ascending) in fv_node, features
 * fv_feat[fv_off[j] .. fv_off[j+1]) (capacities n, n + 1, n). */
orbx_status orbx_vocabulary_transform(orbx_vocabulary* v, const uint8_t* desc, int32_t n,
                                      int32_t levelsup, int32_t* word, int32_t* node,
                                      uint32_t* bow_word, double* bow_value, int32_t* bow_n,
                                      uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                                      int32_t* fv_n);

/* The tree descent alone for n device-resident descriptors (e.g. a whole batch of frames),
 * on the caller's stream: d_word / d_node (n entries each) in device memory. */
orbx_status orbx_vocabulary_transform_device(orbx_vocabulary* v, const uint8_t* d_desc,
                                             int32_t n, int32_t levelsup, int32_t* d_word,
                                             int32_t* d_node, void* stream);

/* L1Scoring::score of two BowVectors (word ids ascending). */
double orbx_bow_score_l1(const uint32_t* w1, const double* v1, int32_t n1, const uint32_t* w2,
                         const double* v2, int32_t n2);

/* The scoring pass of KeyFrameDatabase::DetectRelocalizationCandidates / DetectLoopCandidates
 * (src/KeyFrameDatabase.cc:220-278, 44-163) for nkf keyframes at once: common[i] = the
 * number of the query's words keyframe i's BowVector holds (mnRelocWords / mnLoopWords, the
 * inverted-file count), score[i] = (float)L1Scoring::score(query, keyframe i) (mRelocScore).
 * Keyframe i's BowVector is words/values [kf_off[i], kf_off[i+1]) (ascending words).  The
 * candidate selection that follows (minCommonWords, covisibility accumulation) reads the
 * Map's covisibility graph and stays with the caller.  Host-pointer version: */
orbx_status orbx_bow_db_score(const uint32_t* qword, const double* qval, int32_t nq, int32_t nkf,
                              const int32_t* kf_off, const uint32_t* word, const double* val,
                              int32_t* common, float* score, int device);
/* Device version (all arrays device memory), on the caller's stream. */
orbx_status orbx_bow_db_score_device(const uint32_t* d_qword, const double* d_qval, int32_t nq,
                                     int32_t nkf, const int32_t* d_kf_off,
                                     const uint32_t* d_word, const double* d_val,
                                     int32_t* d_common, float* d_score, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_VOCAB_H */
