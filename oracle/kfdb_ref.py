"""CPU restatement of KeyFrameDatabase::DetectLoopCandidates /
DetectRelocalizationCandidates (src/KeyFrameDatabase.cpp:96-355).

TEST INFRASTRUCTURE ONLY: the oracle for include/orbslam2_amd/
KeyFrameDatabase.h.  Keyframes are dicts with the reference's fields:
id, bow (dict word -> value), connected (set of keyframe indices),
best_covis (list of keyframe indices, GetBestCovisibilityKeyFrames(10)),
and the query bookkeeping (loop_query, loop_words, loop_score, reloc_query,
reloc_words, reloc_score), mutated as the reference mutates them.  Scores by
bow_ref.bow_score (TemplatedVocabulary::score), rounded to float.
"""
from __future__ import annotations

import numpy as np

import bow_ref

f32 = np.float32


class KeyFrameDatabase:
    def __init__(self, n_words, scoring):
        self.scoring = scoring
        self.inv = [[] for _ in range(n_words)]

    def add(self, kfs, i):
        for w in sorted(kfs[i]["bow"]):
            self.inv[w].append(i)

    def erase(self, kfs, i):
        for w in sorted(kfs[i]["bow"]):
            if i in self.inv[w]:
                self.inv[w].remove(i)

    def detect_loop(self, kfs, q, min_score):
        K = kfs[q]
        shared = []
        for w in sorted(K["bow"]):
            for i in self.inv[w]:
                k = kfs[i]
                if k["loop_query"] != K["id"]:
                    k["loop_words"] = 0
                    if i not in K["connected"]:
                        k["loop_query"] = K["id"]
                        shared.append(i)
                k["loop_words"] += 1
        if not shared:
            return []
        max_common = max(kfs[i]["loop_words"] for i in shared)
        min_common = int(f32(max_common) * f32(0.8))
        scored = []
        for i in shared:
            if kfs[i]["loop_words"] > min_common:
                si = f32(bow_ref.bow_score(self.scoring, K["bow"], kfs[i]["bow"])[0])
                kfs[i]["loop_score"] = si
                if si >= f32(min_score):
                    scored.append((si, i))
        if not scored:
            return []
        acc_list, best_acc = [], f32(min_score)
        for si, i in scored:
            best, acc, best_i = si, si, i
            for j in kfs[i]["best_covis"]:
                k2 = kfs[j]
                if k2["loop_query"] == K["id"] and k2["loop_words"] > min_common:
                    acc = f32(acc + k2["loop_score"])
                    if k2["loop_score"] > best:
                        best_i, best = j, k2["loop_score"]
            acc_list.append((acc, best_i))
            if acc > best_acc:
                best_acc = acc
        return _retain(acc_list, f32(f32(0.75) * best_acc))

    def detect_reloc(self, kfs, fbow, fid):
        shared = []
        for w in sorted(fbow):
            for i in self.inv[w]:
                k = kfs[i]
                if k["reloc_query"] != fid:
                    k["reloc_words"] = 0
                    k["reloc_query"] = fid
                    shared.append(i)
                k["reloc_words"] += 1
        if not shared:
            return []
        max_common = max(kfs[i]["reloc_words"] for i in shared)
        min_common = int(f32(max_common) * f32(0.8))
        scored = []
        for i in shared:
            if kfs[i]["reloc_words"] > min_common:
                si = f32(bow_ref.bow_score(self.scoring, fbow, kfs[i]["bow"])[0])
                kfs[i]["reloc_score"] = si
                scored.append((si, i))
        if not scored:
            return []
        acc_list, best_acc = [], f32(0)
        for si, i in scored:
            best, acc, best_i = si, si, i
            for j in kfs[i]["best_covis"]:
                k2 = kfs[j]
                if k2["reloc_query"] != fid:
                    continue
                acc = f32(acc + k2["reloc_score"])
                if k2["reloc_score"] > best:
                    best_i, best = j, k2["reloc_score"]
            acc_list.append((acc, best_i))
            if acc > best_acc:
                best_acc = acc
        return _retain(acc_list, f32(f32(0.75) * best_acc))


def _retain(acc_list, min_keep):
    out, seen = [], set()
    for acc, i in acc_list:
        if acc > min_keep and i not in seen:
            out.append(i)
            seen.add(i)
    return out
