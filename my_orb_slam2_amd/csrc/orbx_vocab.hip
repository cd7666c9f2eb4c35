// orbx_vocab.hip — DBoW2 vocabulary (TemplatedVocabulary<FORB::TDescriptor, FORB>) on gfx950.
//
// The tree lives in HBM as structure-of-arrays: node descriptors (32 B each), the children
// as CSR (in file order: the reference's children vectors), and the word id of every node.
// k_transform descends one descriptor per lane: at each level the k children are compared
// with XOR + v_bcnt and the FIRST minimum wins (`if(d < best_d)`, TemplatedVocabulary.h:1243),
// the node at level L - levelsup is recorded for the FeatureVector.  A k=10, L=6 vocabulary
// (1.1 M nodes, 35 MB) stays L2/MALL-resident across frames.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/orbx_vocab.h"
#include "orbx_host.h"

using namespace orbx;

namespace {

struct HostNode {
    int parent = 0, word_id = 0;   // Node(): word_id(0) (TemplatedVocabulary.h:316)
    double weight = 0;
    uint8_t desc[32] = {0};
};

__device__ __forceinline__ int hamming32(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup) (:1224-1256).
__global__ __launch_bounds__(256) void k_transform(const uint8_t* __restrict__ desc, int n,
                                                   const uint4* __restrict__ ndesc,
                                                   const int32_t* __restrict__ coff,
                                                   const int32_t* __restrict__ child,
                                                   const int32_t* __restrict__ nword,
                                                   int nid_level, int max_depth, int leaf_ids,
                                                   int32_t* __restrict__ oword,
                                                   int32_t* __restrict__ onode) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* f = (const uint4*)(desc + 32 * (size_t)i);
    const uint4 f0 = f[0], f1 = f[1];
    int nid = nid_level <= 0 ? 0 : -1;
    int id = 0;
    for (int level = 1; level <= max_depth; ++level) {
        const int c0 = coff[id], c1 = coff[id + 1];
        if (c0 >= c1) break;   // leaf (Node::isLeaf: no children)
        int best = child[c0];
        int bd = hamming32(f0, f1, ndesc[2 * best], ndesc[2 * best + 1]);
        for (int c = c0 + 1; c < c1; ++c) {
            const int cid = child[c];
            const int d = hamming32(f0, f1, ndesc[2 * cid], ndesc[2 * cid + 1]);
            if (d < bd) { bd = d; best = cid; }
        }
        id = best;
        if (level == nid_level) nid = id;
    }
    oword[i] = leaf_ids ? id : nword[id];
    onode[i] = nid < 0 ? id : nid;   // a leaf above level L-levelsup: the reference leaves nid unset
}

// BoW database scoring: one wave per keyframe.  Lanes binary-search the keyframe's words in
// the query (LDS), the matched terms fabs(v-w) - fabs(v) - fabs(w) land in LDS in word order
// and lane 0 adds them in that order (L1Scoring::score's sequential double sum; unmatched
// positions are skipped, which adds nothing to the sum).
__global__ __launch_bounds__(256) void k_bow_score(const uint32_t* __restrict__ qword,
                                                   const double* __restrict__ qval, int nq,
                                                   int nkf, const int32_t* __restrict__ kf_off,
                                                   const uint32_t* __restrict__ word,
                                                   const double* __restrict__ val,
                                                   int32_t* __restrict__ common,
                                                   float* __restrict__ score) {
    extern __shared__ uint8_t sm[];
    uint32_t* qw = (uint32_t*)sm;                          // nq
    double* qv = (double*)(sm + ((4 * (size_t)nq + 7) & ~(size_t)7));
    double* term = qv + nq + 64 * (threadIdx.x >> 6);      // 64 per wave
    for (int i = threadIdx.x; i < nq; i += 256) {
        qw[i] = qword[i];
        qv[i] = qval[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int kf = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kf >= nkf) return;
    const int o0 = kf_off[kf], o1 = kf_off[kf + 1];
    int cnt = 0;
    double s = 0;
    for (int base = o0; base < o1; base += 64) {
        const int p = base + lane;
        double t = 0;
        bool hit = false;
        if (p < o1) {
            const uint32_t w = word[p];
            int lo = 0, hi = nq;   // lower_bound in the query's words
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (qw[mid] < w) lo = mid + 1; else hi = mid;
            }
            if (lo < nq && qw[lo] == w) {
                const double vi = qv[lo], wi = val[p];
                t = fabs(vi - wi) - fabs(vi) - fabs(wi);
                hit = true;
            }
        }
        term[lane] = t;
        const uint64_t m = __ballot(hit);
        cnt += __popcll(m);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane == 0) {
            uint64_t mm = m;
            while (mm) {
                const int j = __builtin_ctzll(mm);
                mm &= mm - 1;
                s += term[j];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane == 0) {
        common[kf] = cnt;
        score[kf] = (float)(-s / 2.0);
    }
}

}  // namespace

struct orbx_vocabulary {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0;
    int n_nodes = 0, n_words = 0, max_depth = 0;
    std::vector<HostNode> nodes;
    std::vector<int32_t> coff, child;
    hipStream_t stream = nullptr;
    DevBuf d_ndesc, d_coff, d_child, d_word, d_in, d_out;
    std::mutex mu;
};

extern "C" {

orbx_status orbx_vocabulary_load_text(const char* path, int device, orbx_vocabulary** out) {
    if (!path || !out || device < 0) return ORBX_ERR_INVALID;
    *out = nullptr;
    std::ifstream f(path);
    if (!f.is_open()) return ORBX_ERR_INVALID;
    auto* v = new orbx_vocabulary();
    v->device = device;
    std::string s;
    std::getline(f, s);
    std::stringstream ss(s);
    ss >> v->k >> v->L >> v->scoring >> v->weighting;
    if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || v->scoring < 0 || v->scoring > 5 ||
        v->weighting < 0 || v->weighting > 3) {
        delete v;
        return ORBX_ERR_INVALID;
    }
    std::vector<std::vector<int>> children(1);
    v->nodes.resize(1);
    std::string line;
    while (std::getline(f, line)) {
        if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
        std::stringstream sn(line);
        const int nid = (int)v->nodes.size();
        HostNode nd;
        int pid = 0, isleaf = 0;
        sn >> pid >> isleaf;
        if (pid < 0 || pid >= nid) {   // parents precede children in the file format
            delete v;
            return ORBX_ERR_INVALID;
        }
        nd.parent = pid;
        for (int i = 0; i < 32; ++i) {   // FORB::fromString
            int b;
            sn >> b;
            if (!sn.fail()) nd.desc[i] = (uint8_t)b;
        }
        sn >> nd.weight;
        if (isleaf > 0) nd.word_id = v->n_words++;
        v->nodes.push_back(nd);
        children.emplace_back();
        children[pid].push_back(nid);
    }
    v->n_nodes = (int)v->nodes.size();
    v->coff.assign(v->n_nodes + 1, 0);
    for (int i = 0; i < v->n_nodes; ++i) {
        v->coff[i + 1] = v->coff[i] + (int)children[i].size();
        v->child.insert(v->child.end(), children[i].begin(), children[i].end());
    }
    std::vector<int> depth(v->n_nodes, 0);
    for (int i = 1; i < v->n_nodes; ++i) {
        depth[i] = depth[v->nodes[i].parent] + 1;
        v->max_depth = std::max(v->max_depth, depth[i]);
    }
    std::vector<uint8_t> nd(32 * (size_t)v->n_nodes);
    std::vector<int32_t> nw(v->n_nodes);
    for (int i = 0; i < v->n_nodes; ++i) {
        std::memcpy(&nd[32 * (size_t)i], v->nodes[i].desc, 32);
        nw[i] = v->nodes[i].word_id;
    }
    if (!HIPOK(hipSetDevice(device)) ||
        !HIPOK(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking)) ||
        !v->d_ndesc.ensure(nd.size()) || !v->d_coff.ensure(4 * v->coff.size()) ||
        !v->d_child.ensure(4 * std::max<size_t>(v->child.size(), 1)) ||
        !v->d_word.ensure(4 * nw.size()) ||
        !HIPOK(hipMemcpy(v->d_ndesc.p, nd.data(), nd.size(), hipMemcpyHostToDevice)) ||
        !HIPOK(hipMemcpy(v->d_coff.p, v->coff.data(), 4 * v->coff.size(), hipMemcpyHostToDevice)) ||
        (!v->child.empty() &&
         !HIPOK(hipMemcpy(v->d_child.p, v->child.data(), 4 * v->child.size(), hipMemcpyHostToDevice))) ||
        !HIPOK(hipMemcpy(v->d_word.p, nw.data(), 4 * nw.size(), hipMemcpyHostToDevice))) {
        orbx_vocabulary_destroy(v);
        return ORBX_ERR_DEVICE;
    }
    *out = v;
    return ORBX_OK;
}

orbx_status orbx_vocabulary_destroy(orbx_vocabulary* v) {
    if (!v) return ORBX_ERR_INVALID;
    (void)hipSetDevice(v->device);
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    for (DevBuf* b : {&v->d_ndesc, &v->d_coff, &v->d_child, &v->d_word, &v->d_in, &v->d_out})
        b->release();
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
    return ORBX_OK;
}

orbx_status orbx_vocabulary_info(const orbx_vocabulary* v, int32_t* k, int32_t* L,
                                 int32_t* scoring, int32_t* weighting, int32_t* n_nodes,
                                 int32_t* n_words) {
    if (!v) return ORBX_ERR_INVALID;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    return ORBX_OK;
}

orbx_status orbx_vocabulary_transform_device(orbx_vocabulary* v, const uint8_t* d_desc,
                                             int32_t n, int32_t levelsup, int32_t* d_word,
                                             int32_t* d_node, void* stream) {
    if (!v || n < 0 || (n > 0 && (!d_desc || !d_word || !d_node))) return ORBX_ERR_INVALID;
    if ((uintptr_t)d_desc & 15) return ORBX_ERR_INVALID;
    if (n == 0 || v->n_nodes <= 1) return ORBX_OK;
    if (!HIPOK(hipSetDevice(v->device))) return ORBX_ERR_DEVICE;
    hipLaunchKernelGGL(k_transform, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       d_desc, n, v->d_ndesc.as<uint4>(), v->d_coff.as<int32_t>(),
                       v->d_child.as<int32_t>(), v->d_word.as<int32_t>(), v->L - levelsup,
                       v->max_depth, 0, d_word, d_node);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_vocabulary_transform(orbx_vocabulary* v, const uint8_t* desc, int32_t n,
                                      int32_t levelsup, int32_t* word, int32_t* node,
                                      uint32_t* bow_word, double* bow_value, int32_t* bow_n,
                                      uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                                      int32_t* fv_n) {
    if (!v || n < 0 || (n > 0 && !desc) || !bow_word || !bow_value || !bow_n || !fv_node ||
        !fv_off || !fv_feat || !fv_n)
        return ORBX_ERR_INVALID;
    *bow_n = 0;
    *fv_n = 0;
    fv_off[0] = 0;
    if (v->n_nodes <= 1) return ORBX_OK;   // empty(): TemplatedVocabulary.h:1134
    std::lock_guard<std::mutex> lk(v->mu);
    if (!HIPOK(hipSetDevice(v->device))) return ORBX_ERR_DEVICE;
    std::vector<int32_t> leaf(n), nd(n);
    if (n > 0) {
        if (!v->d_in.ensure(32 * (size_t)n) || !v->d_out.ensure(8 * (size_t)n)) return ORBX_ERR_DEVICE;
        if (!HIPOK(hipMemcpyAsync(v->d_in.p, desc, 32 * (size_t)n, hipMemcpyHostToDevice, v->stream)))
            return ORBX_ERR_DEVICE;
        // the final node of every descriptor (its word id and weight are looked up below)
        hipLaunchKernelGGL(k_transform, dim3((n + 255) / 256), dim3(256), 0, v->stream,
                           v->d_in.as<uint8_t>(), n, v->d_ndesc.as<uint4>(), v->d_coff.as<int32_t>(),
                           v->d_child.as<int32_t>(), v->d_word.as<int32_t>(), v->L - levelsup,
                           v->max_depth, 1, v->d_out.as<int32_t>(), v->d_out.as<int32_t>() + n);
        if (!HIPOK(hipGetLastError()) ||
            !HIPOK(hipMemcpyAsync(leaf.data(), v->d_out.p, 4 * (size_t)n, hipMemcpyDeviceToHost, v->stream)) ||
            !HIPOK(hipMemcpyAsync(nd.data(), v->d_out.as<int32_t>() + n, 4 * (size_t)n,
                                  hipMemcpyDeviceToHost, v->stream)) ||
            !HIPOK(hipStreamSynchronize(v->stream)))
            return ORBX_ERR_DEVICE;
    }
    // BowVector / FeatureVector in feature order (:1147-1196): word_id / weight of the final
    // node (:1255-1256); stopped words (weight <= 0) enter neither vector
    std::map<uint32_t, double> bow;
    std::map<uint32_t, std::vector<int>> fv;
    const bool tf = v->weighting == 0 || v->weighting == 1;
    for (int i = 0; i < n; ++i) {
        const HostNode& hn = v->nodes[leaf[i]];
        if (word) word[i] = hn.word_id;
        if (node) node[i] = nd[i];
        if (hn.weight > 0) {
            if (tf) bow[(uint32_t)hn.word_id] += hn.weight;      // BowVector::addWeight
            else bow.emplace((uint32_t)hn.word_id, hn.weight);   // BowVector::addIfNotExist
            fv[(uint32_t)nd[i]].push_back(i);                    // FeatureVector::addFeature
        }
    }
    const bool must = v->scoring != 5;   // every ScoringObject but DotProduct normalizes
    if (tf && !bow.empty() && !must) {
        const double cnt = (double)bow.size();
        for (auto& kv : bow) kv.second /= cnt;
    }
    if (must) {   // BowVector::normalize (BowVector.cpp:62-84): L2 for L2_NORM, else L1
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
    for (auto& kv : fv) {
        fv_node[j] = kv.first;
        for (int fi : kv.second) fv_feat[e++] = fi;
        fv_off[++j] = e;
    }
    *fv_n = j;
    return ORBX_OK;
}

orbx_status orbx_bow_db_score_device(const uint32_t* d_qword, const double* d_qval, int32_t nq,
                                     int32_t nkf, const int32_t* d_kf_off,
                                     const uint32_t* d_word, const double* d_val,
                                     int32_t* d_common, float* d_score, void* stream) {
    if (nq < 0 || nkf < 0 || (nkf > 0 && (!d_kf_off || !d_common || !d_score)) ||
        (nq > 0 && (!d_qword || !d_qval)))
        return ORBX_ERR_INVALID;
    const size_t lds = ((4 * (size_t)nq + 7) & ~(size_t)7) + 8 * ((size_t)nq + 256);
    if (lds > 64 * 1024) return ORBX_ERR_UNSUPPORTED;   // query BowVector up to ~5400 words
    if (nkf == 0) return ORBX_OK;
    hipLaunchKernelGGL(k_bow_score, dim3((nkf + 3) / 4), dim3(256), lds, (hipStream_t)stream,
                       d_qword, d_qval, nq, nkf, d_kf_off, d_word, d_val, d_common, d_score);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_bow_db_score(const uint32_t* qword, const double* qval, int32_t nq, int32_t nkf,
                              const int32_t* kf_off, const uint32_t* word, const double* val,
                              int32_t* common, float* score, int device) {
    if (nq < 0 || nkf < 0 || (nkf > 0 && (!kf_off || !common || !score))) return ORBX_ERR_INVALID;
    if (nkf == 0) return ORBX_OK;
    const int nw = kf_off[nkf] - kf_off[0];
    if (nw < 0 || (nw > 0 && (!word || !val)) || (nq > 0 && (!qword || !qval)))
        return ORBX_ERR_INVALID;
    if (!HIPOK(hipSetDevice(device))) return ORBX_ERR_DEVICE;
    std::vector<int32_t> rel(nkf + 1);
    for (int i = 0; i <= nkf; ++i) rel[i] = kf_off[i] - kf_off[0];
    const size_t bytes = 4 * (size_t)nq + 8 * (size_t)nq + 4 * rel.size() + 4 * (size_t)nw +
                         8 * (size_t)nw + 8 * (size_t)nkf + 64 * 6;
    DevBuf buf;
    if (!buf.ensure(bytes)) return ORBX_ERR_DEVICE;
    uint8_t* b = buf.as<uint8_t>();
    size_t o = 0;
    auto put = [&](const void* src, size_t n) {
        uint8_t* d = b + o;
        o = (o + n + 63) & ~(size_t)63;
        if (n && src && !HIPOK(hipMemcpy(d, src, n, hipMemcpyHostToDevice))) return (uint8_t*)nullptr;
        return d;
    };
    uint8_t* dqv = put(qval, 8 * (size_t)nq);
    uint8_t* dqw = put(qword, 4 * (size_t)nq);
    uint8_t* dv = put(nw ? val + kf_off[0] : nullptr, 8 * (size_t)nw);
    uint8_t* dw = put(nw ? word + kf_off[0] : nullptr, 4 * (size_t)nw);
    uint8_t* doff = put(rel.data(), 4 * rel.size());
    uint8_t* dsc = put(nullptr, 4 * (size_t)nkf);
    uint8_t* dcm = put(nullptr, 4 * (size_t)nkf);
    orbx_status s = ORBX_ERR_DEVICE;
    if (dqv && dqw && dv && dw && doff) {
        s = orbx_bow_db_score_device((uint32_t*)dqw, (double*)dqv, nq, nkf, (int32_t*)doff,
                                     (uint32_t*)dw, (double*)dv, (int32_t*)dcm, (float*)dsc,
                                     nullptr);
        if (s == ORBX_OK &&
            (!HIPOK(hipMemcpy(common, dcm, 4 * (size_t)nkf, hipMemcpyDeviceToHost)) ||
             !HIPOK(hipMemcpy(score, dsc, 4 * (size_t)nkf, hipMemcpyDeviceToHost))))
            s = ORBX_ERR_DEVICE;
    }
    buf.release();
    return s;
}

double orbx_bow_score_l1(const uint32_t* w1, const double* v1, int32_t n1, const uint32_t* w2,
                         const double* v2, int32_t n2) {
    double score = 0;
    int i = 0, j = 0;
    while (i < n1 && j < n2) {
        const double vi = v1[i], wi = v2[j];
        if (w1[i] == w2[j]) {
            score += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
            ++i;
            ++j;
        } else if (w1[i] < w2[j]) {
            while (i < n1 && w1[i] < w2[j]) ++i;   // v1.lower_bound(v2_it->first)
        } else {
            while (j < n2 && w2[j] < w1[i]) ++j;
        }
    }
    return -score / 2.0;
}

}  // extern "C"
