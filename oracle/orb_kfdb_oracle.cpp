// orb_kfdb_oracle.cpp — CPU restatement of ORB_SLAM2::KeyFrameDatabase
// (src/KeyFrameDatabase.cc), TEST INFRASTRUCTURE ONLY (the checker of the GPU keyframe
// database, my_orb_slam2_amd/csrc/orbx_kfdb.hip).
//
// Statement by statement: the inverted file is a list of keyframes per word in add order
// (:40-46, erase :48-67), and the per-query state lives on the keyframe objects exactly as in
// include/KeyFrame.h:147-153 (mnLoopQuery, mnLoopWords, mLoopScore, mnRelocQuery,
// mnRelocWords, mRelocScore).  Keyframes are identified by their add index (the GPU's slot);
// std::set<KeyFrame*> becomes std::set<int> (only membership is used).  The similarity is
// DBoW2's L1Scoring::score (oracle_bow_score_l1, ScoringObject.cpp:23-67), cast to float as
// `float si = mpVoc->score(...)`.
//
// Conventions where the reference is undefined (same as include/orbx_kfdb.h): mRelocScore
// starts at 0 (uninitialised in KeyFrame.cc:35's initialiser list), and each detect call
// gets a fresh query id (F->mnId / pKF->mnId, never 0, which the ctor gives mn*Query).
#include <cstdint>
#include <cstring>
#include <list>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

extern "C" double oracle_bow_score_l1(const uint32_t* w1, const double* v1, int n1,
                                      const uint32_t* w2, const double* v2, int n2);

namespace {

struct OKeyFrame {
    std::vector<uint32_t> words;     // mBowVec (ascending word ids)
    std::vector<double> values;
    std::vector<int> ordered;        // mvpOrderedConnectedKeyFrames (weight-descending)
    unsigned long mnLoopQuery = 0;   // KeyFrame.cc:35
    int mnLoopWords = 0;
    float mLoopScore = 0.f;
    unsigned long mnRelocQuery = 0;
    int mnRelocWords = 0;
    float mRelocScore = 0.f;         // convention (uninitialised in the reference)

    // KeyFrame::GetBestCovisibilityKeyFrames (KeyFrame.cc:178-186)
    std::vector<int> best_covisibles(int N) const {
        if ((int)ordered.size() < N) return ordered;
        return std::vector<int>(ordered.begin(), ordered.begin() + N);
    }
};

struct ODatabase {
    std::vector<OKeyFrame> kfs;                             // by add index (slot)
    std::unordered_map<uint32_t, std::list<int>> inv;       // mvInvertedFile
    unsigned long next_query = 1;
    int covisibles = 10;

    double score(const std::vector<uint32_t>& qw, const std::vector<double>& qv,
                 const OKeyFrame& k) const {
        return oracle_bow_score_l1(qw.data(), qv.data(), (int)qw.size(), k.words.data(),
                                   k.values.data(), (int)k.words.size());
    }

    // KeyFrameDatabase::DetectLoopCandidates (:76-208); `connected` = GetConnectedKeyFrames()
    std::vector<int> detect_loop(const std::vector<uint32_t>& qw, const std::vector<double>& qv,
                                 const std::set<int>& spConnectedKeyFrames, float minScore) {
        const unsigned long id = next_query++;
        std::list<int> lKFsSharingWords;
        for (uint32_t w : qw) {                                           // :89-110
            auto it = inv.find(w);
            if (it == inv.end()) continue;
            for (int i : it->second) {
                OKeyFrame& pKFi = kfs[i];
                if (pKFi.mnLoopQuery != id) {
                    pKFi.mnLoopWords = 0;
                    if (!spConnectedKeyFrames.count(i)) {
                        pKFi.mnLoopQuery = id;
                        lKFsSharingWords.push_back(i);
                    }
                }
                pKFi.mnLoopWords++;
            }
        }
        if (lKFsSharingWords.empty()) return {};                          // :113-114
        std::list<std::pair<float, int>> lScoreAndMatch;
        int maxCommonWords = 0;                                           // :120-125
        for (int i : lKFsSharingWords)
            if (kfs[i].mnLoopWords > maxCommonWords) maxCommonWords = kfs[i].mnLoopWords;
        int minCommonWords = maxCommonWords * 0.8f;                       // :127
        for (int i : lKFsSharingWords) {                                  // :133-147
            OKeyFrame& pKFi = kfs[i];
            if (pKFi.mnLoopWords > minCommonWords) {
                float si = (float)score(qw, qv, pKFi);
                pKFi.mLoopScore = si;
                if (si >= minScore) lScoreAndMatch.push_back(std::make_pair(si, i));
            }
        }
        if (lScoreAndMatch.empty()) return {};                            // :149-150
        std::list<std::pair<float, int>> lAccScoreAndMatch;
        float bestAccScore = minScore;
        for (auto& it : lScoreAndMatch) {                                 // :159-184
            std::vector<int> vpNeighs = kfs[it.second].best_covisibles(covisibles);
            float bestScore = it.first;
            float accScore = it.first;
            int pBestKF = it.second;
            for (int n2 : vpNeighs) {
                const OKeyFrame& pKF2 = kfs[n2];
                if (pKF2.mnLoopQuery == id && pKF2.mnLoopWords > minCommonWords) {
                    accScore += pKF2.mLoopScore;
                    if (pKF2.mLoopScore > bestScore) {
                        pBestKF = n2;
                        bestScore = pKF2.mLoopScore;
                    }
                }
            }
            lAccScoreAndMatch.push_back(std::make_pair(accScore, pBestKF));
            if (accScore > bestAccScore) bestAccScore = accScore;
        }
        float minScoreToRetain = 0.75f * bestAccScore;                    // :187
        std::set<int> spAlreadyAddedKF;
        std::vector<int> vpLoopCandidates;
        for (auto& it : lAccScoreAndMatch) {                              // :193-204
            if (it.first > minScoreToRetain) {
                const int pKFi = it.second;
                if (!spAlreadyAddedKF.count(pKFi)) {
                    vpLoopCandidates.push_back(pKFi);
                    spAlreadyAddedKF.insert(pKFi);
                }
            }
        }
        return vpLoopCandidates;
    }

    // KeyFrameDatabase::DetectRelocalizationCandidates (:220-337)
    std::vector<int> detect_reloc(const std::vector<uint32_t>& qw, const std::vector<double>& qv) {
        const unsigned long id = next_query++;
        std::list<int> lKFsSharingWords;
        for (uint32_t w : qw) {                                           // :230-245
            auto it = inv.find(w);
            if (it == inv.end()) continue;
            for (int i : it->second) {
                OKeyFrame& pKFi = kfs[i];
                if (pKFi.mnRelocQuery != id) {
                    pKFi.mnRelocWords = 0;
                    pKFi.mnRelocQuery = id;
                    lKFsSharingWords.push_back(i);
                }
                pKFi.mnRelocWords++;
            }
        }
        if (lKFsSharingWords.empty()) return {};                          // :247-248
        int maxCommonWords = 0;                                           // :251-257
        for (int i : lKFsSharingWords)
            if (kfs[i].mnRelocWords > maxCommonWords) maxCommonWords = kfs[i].mnRelocWords;
        int minCommonWords = maxCommonWords * 0.8f;                       // :259
        std::list<std::pair<float, int>> lScoreAndMatch;
        for (int i : lKFsSharingWords) {                                  // :266-277
            OKeyFrame& pKFi = kfs[i];
            if (pKFi.mnRelocWords > minCommonWords) {
                float si = (float)score(qw, qv, pKFi);
                pKFi.mRelocScore = si;
                lScoreAndMatch.push_back(std::make_pair(si, i));
            }
        }
        if (lScoreAndMatch.empty()) return {};                            // :279-280
        std::list<std::pair<float, int>> lAccScoreAndMatch;
        float bestAccScore = 0;
        for (auto& it : lScoreAndMatch) {                                 // :289-314
            std::vector<int> vpNeighs = kfs[it.second].best_covisibles(covisibles);
            float bestScore = it.first;
            float accScore = bestScore;
            int pBestKF = it.second;
            for (int n2 : vpNeighs) {
                const OKeyFrame& pKF2 = kfs[n2];
                if (pKF2.mnRelocQuery != id) continue;
                accScore += pKF2.mRelocScore;
                if (pKF2.mRelocScore > bestScore) {
                    pBestKF = n2;
                    bestScore = pKF2.mRelocScore;
                }
            }
            lAccScoreAndMatch.push_back(std::make_pair(accScore, pBestKF));
            if (accScore > bestAccScore) bestAccScore = accScore;
        }
        float minScoreToRetain = 0.75f * bestAccScore;                    // :318
        std::set<int> spAlreadyAddedKF;
        std::vector<int> vpRelocCandidates;
        for (auto& it : lAccScoreAndMatch) {                              // :322-334
            const float& si = it.first;
            if (si > minScoreToRetain) {
                const int pKFi = it.second;
                if (!spAlreadyAddedKF.count(pKFi)) {
                    vpRelocCandidates.push_back(pKFi);
                    spAlreadyAddedKF.insert(pKFi);
                }
            }
        }
        return vpRelocCandidates;
    }
};

int copy_out(const std::vector<int>& v, int32_t* out, int cap) {
    for (size_t i = 0; i < v.size() && (int)i < cap; ++i) out[i] = v[i];
    return (int)v.size();
}

}  // namespace

extern "C" {

void* oracle_kfdb_create(int covisibles) {
    ODatabase* d = new ODatabase();
    d->covisibles = covisibles;
    return d;
}

void oracle_kfdb_destroy(void* h) { delete (ODatabase*)h; }

// KeyFrameDatabase::add (:40-46)
int oracle_kfdb_add(void* h, const uint32_t* w, const double* v, int n) {
    ODatabase* d = (ODatabase*)h;
    OKeyFrame k;
    k.words.assign(w, w + n);
    k.values.assign(v, v + n);
    d->kfs.push_back(k);
    const int slot = (int)d->kfs.size() - 1;
    for (int j = 0; j < n; ++j) d->inv[w[j]].push_back(slot);
    return slot;
}

// KeyFrameDatabase::erase (:48-67)
void oracle_kfdb_erase(void* h, int slot) {
    ODatabase* d = (ODatabase*)h;
    const OKeyFrame& k = d->kfs[slot];
    for (uint32_t w : k.words) {
        std::list<int>& l = d->inv[w];
        for (auto it = l.begin(); it != l.end(); ++it)
            if (*it == slot) {
                l.erase(it);
                break;
            }
    }
}

// KeyFrameDatabase::clear (:69-73); the slots restart at 0 like the GPU database
void oracle_kfdb_clear(void* h) {
    ODatabase* d = (ODatabase*)h;
    d->inv.clear();
    d->kfs.clear();
}

void oracle_kfdb_set_covisibles(void* h, int slot, const int32_t* nb, int n) {
    ODatabase* d = (ODatabase*)h;
    d->kfs[slot].ordered.assign(nb, nb + n);
}

int oracle_kfdb_detect_reloc(void* h, const uint32_t* qw, const double* qv, int nq, int32_t* out,
                             int cap) {
    ODatabase* d = (ODatabase*)h;
    return copy_out(d->detect_reloc(std::vector<uint32_t>(qw, qw + nq),
                                    std::vector<double>(qv, qv + nq)),
                    out, cap);
}

int oracle_kfdb_detect_loop(void* h, const uint32_t* qw, const double* qv, int nq,
                            const int32_t* conn, int nc, float min_score, int32_t* out, int cap) {
    ODatabase* d = (ODatabase*)h;
    return copy_out(d->detect_loop(std::vector<uint32_t>(qw, qw + nq),
                                   std::vector<double>(qv, qv + nq),
                                   std::set<int>(conn, conn + nc), min_score),
                    out, cap);
}

}  // extern "C"
