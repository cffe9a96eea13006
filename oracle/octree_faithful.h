// octree_faithful.h -- DistributeOctTree with the REFERENCE'S allocation
// pattern, for the H2 measurement only (tools/h2_tiebreak.py, DESIGN.md §5;
// TEST INFRASTRUCTURE ONLY, included by orbref.cpp).
//
// The reference sorts pair<int, ExtractorNode*> (src/ORBextractor.cpp:690),
// so equal-size nodes are ordered by the heap address of their std::list
// node.  This restatement keeps everything that decides those addresses:
// the node type's layout (ExtractorNode: vector<cv::KeyPoint> of 28-byte
// keypoints, four cv::Point2i, a list iterator and a bool;
// include/ORBextractor.h:32-45), the std::list push_back / push_front /
// erase sequence, DivideNode's four reserve(vKeys.size()) calls
// (ORBextractor.cpp:483-539), the vector copies made by push_front, the
// destruction order of the four local children, vSizeAndPointerToNode and its
// copy (:561, :594, :681-743).  Allocation goes through Alloc:
//   * RealAlloc -- the process's glibc malloc (the reference's mechanism, in
//     whatever heap state this process is in);
//   * ModelAlloc -- a deterministic model of glibc for this sequence: chunk
//     sizes as glibc rounds them, per-size LIFO reuse of freed chunks (the
//     tcache / fastbin behaviour; larger freed chunks are also reused by exact
//     size, no splitting or coalescing), otherwise carved from a top chunk at
//     increasing addresses starting from an empty heap.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <list>
#include <map>
#include <memory>
#include <utility>
#include <vector>

namespace h2 {

struct KP28 {  // cv::KeyPoint (OpenCV 2.4): pt, size, angle, response, octave, class_id
    float x, y, size, angle, response;
    int octave, class_id;
};
struct Pt {
    int x, y;
};

// ---- allocators ----------------------------------------------------------
struct ModelHeap {
    uintptr_t top = 0x10000;
    std::map<size_t, std::vector<uintptr_t>> free_lists;  // chunk size -> LIFO
    std::map<uintptr_t, size_t> live;                      // fake address -> chunk size
    static size_t chunk(size_t req) { return std::max<size_t>(32, (req + 8 + 15) & ~size_t(15)); }
    uintptr_t alloc(size_t req) {
        const size_t c = chunk(req);
        auto& fl = free_lists[c];
        uintptr_t a;
        if (!fl.empty()) {
            a = fl.back();
            fl.pop_back();
        } else {
            a = top + 16;  // user pointer after the chunk header
            top += c;
        }
        live[a] = c;
        return a;
    }
    void release(uintptr_t a) {
        auto it = live.find(a);
        if (it == live.end()) return;
        free_lists[it->second].push_back(a);
        live.erase(it);
    }
};

// Every allocation is real (the containers need real memory); `addr` maps a
// real pointer to the address used for ordering: itself (real mode) or the
// model heap's address for the same allocation.
struct Heap {
    bool model = false;
    ModelHeap m;
    std::map<const void*, uintptr_t> addr_of;
    void on_alloc(const void* p, size_t n) {
        if (model) addr_of[p] = m.alloc(n);
    }
    void on_free(const void* p) {
        if (!model) return;
        auto it = addr_of.find(p);
        if (it == addr_of.end()) return;
        m.release(it->second);
        addr_of.erase(it);
    }
    uintptr_t addr(const void* p) const {
        if (!model) return (uintptr_t)p;
        auto it = addr_of.find(p);
        return it == addr_of.end() ? (uintptr_t)p : it->second;
    }
};
extern thread_local Heap* g_heap;

template <class T>
struct TrackAlloc {
    using value_type = T;
    TrackAlloc() = default;
    template <class U>
    TrackAlloc(const TrackAlloc<U>&) {}
    T* allocate(size_t n) {
        T* p = static_cast<T*>(std::malloc(n * sizeof(T)));
        if (g_heap) g_heap->on_alloc(p, n * sizeof(T));
        return p;
    }
    void deallocate(T* p, size_t) {
        if (g_heap) g_heap->on_free(p);
        std::free(p);
    }
    template <class U>
    bool operator==(const TrackAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const TrackAlloc<U>&) const { return false; }
};

struct ExtractorNode;
using NodeList = std::list<ExtractorNode, TrackAlloc<ExtractorNode>>;
struct ExtractorNode {  // include/ORBextractor.h:32-45 field order
    std::vector<KP28, TrackAlloc<KP28>> vKeys;
    Pt UL{}, UR{}, BL{}, BR{};
    NodeList::iterator lit;
    bool bNoMore = false;
    void DivideNode(ExtractorNode& n1, ExtractorNode& n2, ExtractorNode& n3, ExtractorNode& n4) {  // :483-539
        const int halfX = (int)std::ceil((float)(UR.x - UL.x) / 2);
        const int halfY = (int)std::ceil((float)(BR.y - UL.y) / 2);
        n1.UL = UL;
        n1.UR = Pt{UL.x + halfX, UL.y};
        n1.BL = Pt{UL.x, UL.y + halfY};
        n1.BR = Pt{UL.x + halfX, UL.y + halfY};
        n1.vKeys.reserve(vKeys.size());
        n2.UL = n1.UR;
        n2.UR = UR;
        n2.BL = n1.BR;
        n2.BR = Pt{UR.x, UL.y + halfY};
        n2.vKeys.reserve(vKeys.size());
        n3.UL = n1.BL;
        n3.UR = n1.BR;
        n3.BL = BL;
        n3.BR = Pt{n1.BR.x, BL.y};
        n3.vKeys.reserve(vKeys.size());
        n4.UL = n3.UR;
        n4.UR = n2.BR;
        n4.BL = n3.BR;
        n4.BR = BR;
        n4.vKeys.reserve(vKeys.size());
        for (size_t i = 0; i < vKeys.size(); i++) {
            const KP28& kp = vKeys[i];
            if (kp.x < n1.UR.x) {
                if (kp.y < n1.BR.y) n1.vKeys.push_back(kp);
                else n3.vKeys.push_back(kp);
            } else if (kp.y < n1.BR.y) {
                n2.vKeys.push_back(kp);
            } else {
                n4.vKeys.push_back(kp);
            }
        }
        if (n1.vKeys.size() == 1) n1.bNoMore = true;
        if (n2.vKeys.size() == 1) n2.bNoMore = true;
        if (n3.vKeys.size() == 1) n3.bNoMore = true;
        if (n4.vKeys.size() == 1) n4.bNoMore = true;
    }
};

// ORBextractor.cpp:541-770 (keys relative to (minX, minY); class_id carries the
// candidate index); returns the kept candidates in list order
inline std::vector<int> distribute(const std::vector<KP28>& vToDistributeKeys, int minX, int maxX, int minY,
                                   int maxY, int N) {
    using PairV = std::vector<std::pair<int, ExtractorNode*>, TrackAlloc<std::pair<int, ExtractorNode*>>>;
    const Heap* H = g_heap;
    auto less_addr = [H](const std::pair<int, ExtractorNode*>& a, const std::pair<int, ExtractorNode*>& b) {
        if (a.first != b.first) return a.first < b.first;
        return H->addr(a.second) < H->addr(b.second);  // pair<int, ExtractorNode*> order
    };
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    NodeList lNodes;
    std::vector<ExtractorNode*, TrackAlloc<ExtractorNode*>> vpIniNodes;
    vpIniNodes.resize(nIni);
    for (int i = 0; i < nIni; i++) {
        ExtractorNode ni;
        ni.UL = Pt{(int)(hX * static_cast<float>(i)), 0};
        ni.UR = Pt{(int)(hX * static_cast<float>(i + 1)), 0};
        ni.BL = Pt{ni.UL.x, maxY - minY};
        ni.BR = Pt{ni.UR.x, maxY - minY};
        ni.vKeys.reserve(vToDistributeKeys.size());
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (size_t i = 0; i < vToDistributeKeys.size(); i++) {
        const KP28& kp = vToDistributeKeys[i];
        vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
    }
    auto lit = lNodes.begin();
    while (lit != lNodes.end()) {
        if (lit->vKeys.size() == 1) {
            lit->bNoMore = true;
            lit++;
        } else if (lit->vKeys.empty()) {
            lit = lNodes.erase(lit);
        } else {
            lit++;
        }
    }
    bool bFinish = false;
    PairV vSizeAndPointerToNode;
    vSizeAndPointerToNode.reserve(lNodes.size() * 4);
    auto add = [&](ExtractorNode& n, int& nToExpand, PairV& v) {
        if (n.vKeys.size() > 0) {
            lNodes.push_front(n);
            if (n.vKeys.size() > 1) {
                nToExpand++;
                v.push_back(std::make_pair((int)n.vKeys.size(), &lNodes.front()));
                lNodes.front().lit = lNodes.begin();
            }
        }
    };
    while (!bFinish) {
        int prevSize = (int)lNodes.size();
        lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) {
                lit++;
                continue;
            }
            ExtractorNode n1, n2, n3, n4;
            lit->DivideNode(n1, n2, n3, n4);
            add(n1, nToExpand, vSizeAndPointerToNode);
            add(n2, nToExpand, vSizeAndPointerToNode);
            add(n3, nToExpand, vSizeAndPointerToNode);
            add(n4, nToExpand, vSizeAndPointerToNode);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                PairV vPrevSizeAndPointerToNode = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                std::sort(vPrevSizeAndPointerToNode.begin(), vPrevSizeAndPointerToNode.end(), less_addr);
                for (int j = (int)vPrevSizeAndPointerToNode.size() - 1; j >= 0; j--) {
                    ExtractorNode n1, n2, n3, n4;
                    vPrevSizeAndPointerToNode[j].second->DivideNode(n1, n2, n3, n4);
                    int dummy = 0;
                    add(n1, dummy, vSizeAndPointerToNode);
                    add(n2, dummy, vSizeAndPointerToNode);
                    add(n3, dummy, vSizeAndPointerToNode);
                    add(n4, dummy, vSizeAndPointerToNode);
                    lNodes.erase(vPrevSizeAndPointerToNode[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<int> kept;
    for (lit = lNodes.begin(); lit != lNodes.end(); lit++) {  // :751-767
        const auto& vNodeKeys = lit->vKeys;
        const KP28* pKP = &vNodeKeys[0];
        float maxResponse = pKP->response;
        for (size_t k = 1; k < vNodeKeys.size(); k++)
            if (vNodeKeys[k].response > maxResponse) {
                pKP = &vNodeKeys[k];
                maxResponse = vNodeKeys[k].response;
            }
        kept.push_back(pKP->class_id);
    }
    return kept;
}

}  // namespace h2
