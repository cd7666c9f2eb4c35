// orb_vocab_oracle.cpp — CPU restatement of the DBoW2 vocabulary path the matchers depend on
// (TEST INFRASTRUCTURE ONLY).
//
// DBoW2 is vendored in the reference (Thirdparty/DBoW2); restated here:
//   TemplatedVocabulary::loadFromTextFile   TemplatedVocabulary.h:1338-1417
//   TemplatedVocabulary::transform (x3)     TemplatedVocabulary.h:1123-1256
//   BowVector::addWeight/addIfNotExist/normalize   BowVector.cpp:34-84
//   FeatureVector::addFeature               FeatureVector.cpp:31-45
//   L1Scoring::score                        ScoringObject.cpp:23-67
// The real ORBvoc.txt is not in the reference checkout (.MISSING_LARGE_BLOBS); tests use
// synthetic vocabularies in the same text format.  Parity of the restatement is pinned by
// the cross-checks in tests/, not by a run of the reference (PARITY UNPINNED).
//
// Deviation: the reference's `while(!f.eof())` loop turns the empty line after a final
// newline into an extra child of the root with an unread descriptor (undefined contents);
// this loader skips blank lines.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Node {
    int id = 0, parent = 0, word_id = 0;
    double weight = 0;
    std::vector<int> children;
    uint8_t desc[32] = {0};
    bool isLeaf() const { return children.empty(); }   // TemplatedVocabulary.h:328
};

struct Vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<Node> nodes;
    std::vector<int> words;   // word id -> node id
};

int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

}  // namespace

extern "C" {

void* oracle_vocab_load(const char* path) {
    std::ifstream f(path);
    if (!f.is_open()) return nullptr;
    auto* v = new Vocab();
    std::string s;
    std::getline(f, s);
    std::stringstream ss(s);
    ss >> v->k >> v->L >> v->scoring >> v->weighting;
    if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || v->scoring < 0 || v->scoring > 5 ||
        v->weighting < 0 || v->weighting > 3) {
        delete v;
        return nullptr;
    }
    v->nodes.resize(1);
    v->nodes[0].id = 0;
    std::string line;
    while (std::getline(f, line)) {
        if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
        std::stringstream sn(line);
        const int nid = (int)v->nodes.size();
        v->nodes.resize(nid + 1);
        Node& n = v->nodes[nid];
        n.id = nid;
        int pid = 0, isleaf = 0;
        sn >> pid >> isleaf;
        n.parent = pid;
        v->nodes[pid].children.push_back(nid);
        for (int i = 0; i < 32; ++i) {   // FORB::fromString
            int b;
            sn >> b;
            if (!sn.fail()) v->nodes[nid].desc[i] = (uint8_t)b;
        }
        sn >> v->nodes[nid].weight;
        if (isleaf > 0) {
            v->nodes[nid].word_id = (int)v->words.size();
            v->words.push_back(nid);
        }
    }
    return v;
}

void oracle_vocab_free(void* h) { delete (Vocab*)h; }

int oracle_vocab_info(void* h, int32_t* out4) {
    Vocab* v = (Vocab*)h;
    out4[0] = v->k; out4[1] = v->L; out4[2] = v->scoring; out4[3] = v->weighting;
    return (int)v->nodes.size();
}

// transform(feature, word_id, weight, nid, levelsup), TemplatedVocabulary.h:1224-1256, for
// n descriptors; then the BowVector / FeatureVector of transform(features, v, fv, levelsup)
// (:1123-1196).  Outputs: per feature word/nid; bow_word/bow_value (sorted, *bow_n entries);
// the FeatureVector as CSR (fv_node, fv_off, fv_feat).
void oracle_vocab_transform(void* h, const uint8_t* desc, int n, int levelsup, int32_t* word,
                            int32_t* nodeid, int32_t* bow_n, uint32_t* bow_word,
                            double* bow_value, int32_t* fv_n, uint32_t* fv_node, int32_t* fv_off,
                            int32_t* fv_feat) {
    Vocab* v = (Vocab*)h;
    std::map<uint32_t, double> bow;
    std::map<uint32_t, std::vector<int>> fv;
    const int nid_level = v->L - levelsup;
    for (int i = 0; i < n; ++i) {
        const uint8_t* feature = desc + 32 * (size_t)i;
        int nid = nid_level <= 0 ? 0 : -1;
        int final_id = 0, current_level = 0;
        do {
            ++current_level;
            const std::vector<int>& nodes = v->nodes[final_id].children;
            final_id = nodes[0];
            double best_d = hamming(feature, v->nodes[final_id].desc);
            for (size_t c = 1; c < nodes.size(); ++c) {
                const double d = hamming(feature, v->nodes[nodes[c]].desc);
                if (d < best_d) {
                    best_d = d;
                    final_id = nodes[c];
                }
            }
            if (current_level == nid_level) nid = final_id;
        } while (!v->nodes[final_id].isLeaf());
        if (nid < 0) nid = final_id;   // the reference leaves nid unset here (shallow leaf)
        word[i] = v->nodes[final_id].word_id;
        nodeid[i] = nid;
        const double w = v->nodes[final_id].weight;
        if (w > 0) {
            if (v->weighting == 0 || v->weighting == 1) bow[word[i]] += w;   // addWeight
            else bow.emplace((uint32_t)word[i], w);                           // addIfNotExist
            fv[(uint32_t)nid].push_back(i);
        }
    }
    // mustNormalize: every scoring but DOT_PRODUCT, with L2 for L2_NORM, else L1
    const bool must = v->scoring != 5;
    if ((v->weighting == 0 || v->weighting == 1) && !bow.empty() && !must) {
        const double nd = (double)bow.size();
        for (auto& kv : bow) kv.second /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (v->scoring != 1) {
            for (auto& kv : bow) norm += std::fabs(kv.second);
        } else {
            for (auto& kv : bow) norm += kv.second * kv.second;
            norm = std::sqrt(norm);
        }
        if (norm > 0.0)
            for (auto& kv : bow) kv.second /= norm;
    }
    int k = 0;
    for (auto& kv : bow) {
        bow_word[k] = kv.first;
        bow_value[k] = kv.second;
        ++k;
    }
    *bow_n = k;
    int j = 0, e = 0;
    fv_off[0] = 0;
    for (auto& kv : fv) {
        fv_node[j] = kv.first;
        for (int f : kv.second) fv_feat[e++] = f;
        fv_off[++j] = e;
    }
    *fv_n = j;
}

// L1Scoring::score (ScoringObject.cpp:23-67) of two BowVectors (sorted word ids).
double oracle_bow_score_l1(const uint32_t* w1, const double* v1, int n1, const uint32_t* w2,
                           const double* v2, int n2) {
    double score = 0;
    int i = 0, j = 0;
    while (i < n1 && j < n2) {
        const double vi = v1[i], wi = v2[j];
        if (w1[i] == w2[j]) {
            score += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
            ++i;
            ++j;
        } else if (w1[i] < w2[j]) {
            while (i < n1 && w1[i] < w2[j]) ++i;   // lower_bound
        } else {
            while (j < n2 && w2[j] < w1[i]) ++j;
        }
    }
    return -score / 2.0;
}

}  // extern "C"
