"""FewRel / GloVe JSON ingestion, tensorisation and the ``_processed_data`` cache.

Behavioural contract (reference ``util/data_loader.py``):

* FewRel JSON ``{rel: [{"tokens", "h": [name, qid, [[pos..]..]], "t": ...}]}`` (``:62-78``);
  only the first token of the first mention is used (``:160-161``).
* word-vector JSON ``[{"word", "vec"}]`` (``:79-84``); rows are L2-normalised (``:138``);
  ``UNK = V`` and ``BLANK = V + 1`` are appended as all-zero rows (``:124-141``).
* tensorisation (``:143-193``): lower-cased lookups, OOV -> UNK, padding -> BLANK,
  ``length = min(len, L)``, entity positions clamped to ``L-1``, ``pos = j - p + L``,
  PCNN mask segments {0 pad, 1 <= min(p1,p2), 2 <= max, 3 after}.
* cache (``:21-58,197-211``): ``_processed_data/{data}_{word,pos1,pos2,mask,length}.npy``,
  ``{data}_rel2scope.json``, ``{wv}_mat.npy``, ``{wv}_word2id.json``; invalidated only
  when ``word.shape[1] != max_length``.

Differences (documented fixes): a zero GloVe row is left at zero instead of producing
NaN; the ``cuda`` flag is gone (device placement is the engine's job).
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np


def _prefix(path: str) -> str:
    return ".".join(path.split("/")[-1].split(".")[:-1])


class FewRelDataset:
    """Fixed-length int32 arrays for every instance plus the relation scopes."""

    def __init__(self, word: np.ndarray, pos1: np.ndarray, pos2: np.ndarray, mask: np.ndarray,
                 length: np.ndarray, rel2scope: "OrderedDict[str, List[int]]",
                 word_vec_mat: Optional[np.ndarray] = None, word2id: Optional[Dict[str, int]] = None,
                 name: str = "data"):
        self.data_word = np.ascontiguousarray(word, dtype=np.int32)
        self.data_pos1 = np.ascontiguousarray(pos1, dtype=np.int32)
        self.data_pos2 = np.ascontiguousarray(pos2, dtype=np.int32)
        self.data_mask = np.ascontiguousarray(mask, dtype=np.int32)
        self.data_length = np.ascontiguousarray(length, dtype=np.int32)
        self.rel2scope = OrderedDict((k, [int(v[0]), int(v[1])]) for k, v in rel2scope.items())
        self.word_vec_mat = word_vec_mat
        self.word2id = word2id
        self.name = name
        self.max_length = int(self.data_word.shape[1])
        # optional BERT input features (data/bert_tokenize.py): ids / mask / e1 / e2 / length
        self.bert: Optional[Dict[str, np.ndarray]] = None

    # ------------------------------------------------------------------ info
    @property
    def num_instances(self) -> int:
        return int(self.data_word.shape[0])

    @property
    def num_relations(self) -> int:
        return len(self.rel2scope)

    def relations(self) -> List[str]:
        return list(self.rel2scope.keys())

    def scope_array(self) -> np.ndarray:
        """[R, 2] int32 (begin, end) in relation order -- what the device sampler consumes."""
        return np.asarray([self.rel2scope[r] for r in self.rel2scope], dtype=np.int32).reshape(-1, 2)

    def subset_relations(self, rels: List[str], name: Optional[str] = None,
                         part: Optional[Tuple[float, float]] = None) -> "FewRelDataset":
        """Relation-disjoint split helper (train.json is absent: split val.json by relation).
        ``part=(lo, hi)`` keeps only instances [lo, hi) (fractions) of every relation's scope --
        the instance-disjoint split (same relations, disjoint sentences)."""
        idx, scope, i = [], OrderedDict(), 0
        for r in rels:
            b, e = self.rel2scope[r]
            if part is not None:
                n = e - b
                b, e = b + int(round(part[0] * n)), b + int(round(part[1] * n))
            idx.append(np.arange(b, e))
            scope[r] = [i, i + (e - b)]
            i += e - b
        idx = np.concatenate(idx)
        out = FewRelDataset(self.data_word[idx], self.data_pos1[idx], self.data_pos2[idx],
                            self.data_mask[idx], self.data_length[idx], scope,
                            self.word_vec_mat, self.word2id, name or self.name)
        if self.bert is not None:
            out.bert = {k: v[idx] for k, v in self.bert.items()}
        return out

    # -------------------------------------------------------------- tensorise
    @staticmethod
    def build_word_vectors(ori_word_vec: list, case_sensitive: bool = False):
        """GloVe JSON list -> (word2id, L2-normalised [V+2, D] float32 with zero UNK/BLANK)."""
        tot = len(ori_word_vec)
        dim = len(ori_word_vec[0]["vec"])
        mat = np.zeros((tot + 2, dim), dtype=np.float32)
        word2id: Dict[str, int] = {}
        for cur_id, item in enumerate(ori_word_vec):
            w = item["word"] if case_sensitive else item["word"].lower()
            word2id[w] = cur_id
            mat[cur_id, :] = item["vec"]
        norms = np.sqrt((mat[:tot] ** 2).sum(axis=1, keepdims=True))
        np.divide(mat[:tot], norms, out=mat[:tot], where=norms > 0)
        word2id["UNK"] = tot
        word2id["BLANK"] = tot + 1
        return word2id, mat

    @staticmethod
    def tensorize(ori_data: dict, word2id: Dict[str, int], max_length: int,
                  case_sensitive: bool = False):
        unk, blank = word2id["UNK"], word2id["BLANK"]
        L = max_length
        tot = sum(len(v) for v in ori_data.values())
        word = np.full((tot, L), blank, dtype=np.int32)
        pos1 = np.zeros((tot, L), dtype=np.int32)
        pos2 = np.zeros((tot, L), dtype=np.int32)
        mask = np.zeros((tot, L), dtype=np.int32)
        length = np.zeros((tot,), dtype=np.int32)
        rel2scope: "OrderedDict[str, List[int]]" = OrderedDict()
        j_idx = np.arange(L, dtype=np.int32)
        i = 0
        for rel, items in ori_data.items():
            rel2scope[rel] = [i, i]
            for ins in items:
                toks = ins["tokens"]
                if not case_sensitive:
                    toks = [t.lower() for t in toks]
                n = min(len(toks), L)
                get = word2id.get
                word[i, :n] = [get(t, unk) for t in toks[:n]]
                length[i] = n
                p1 = min(int(ins["h"][2][0][0]), L - 1)
                p2 = min(int(ins["t"][2][0][0]), L - 1)
                pos1[i] = j_idx - p1 + L
                pos2[i] = j_idx - p2 + L
                lo, hi = min(p1, p2), max(p1, p2)
                m = np.where(j_idx <= lo, 1, np.where(j_idx <= hi, 2, 3)).astype(np.int32)
                m[j_idx >= n] = 0
                mask[i] = m
                i += 1
            rel2scope[rel][1] = i
        return word, pos1, pos2, mask, length, rel2scope

    # ------------------------------------------------------------------ cache
    @staticmethod
    def _cache_paths(file_name: str, word_vec_file_name: str, processed_dir: str) -> Dict[str, str]:
        p, wp = _prefix(file_name), _prefix(word_vec_file_name)
        j = lambda s: os.path.join(processed_dir, s)
        return {"word": j(p + "_word.npy"), "pos1": j(p + "_pos1.npy"), "pos2": j(p + "_pos2.npy"),
                "mask": j(p + "_mask.npy"), "length": j(p + "_length.npy"),
                "rel2scope": j(p + "_rel2scope.json"), "mat": j(wp + "_mat.npy"),
                "word2id": j(wp + "_word2id.json")}

    @classmethod
    def from_json(cls, file_name: str, word_vec_file_name: str, max_length: int = 40,
                  case_sensitive: bool = False, reprocess: bool = False,
                  processed_dir: str = "_processed_data", verbose: bool = True) -> "FewRelDataset":
        paths = cls._cache_paths(file_name, word_vec_file_name, processed_dir)
        if not reprocess and all(os.path.exists(v) for v in paths.values()):
            word = np.load(paths["word"])
            if word.shape[1] == max_length:
                if verbose:
                    print("Pre-processed files exist. Loading them...")
                with open(paths["rel2scope"]) as f:
                    r2s = json.load(f, object_pairs_hook=OrderedDict)
                with open(paths["word2id"]) as f:
                    w2i = json.load(f)
                return cls(word, np.load(paths["pos1"]), np.load(paths["pos2"]), np.load(paths["mask"]),
                           np.load(paths["length"]), r2s, np.load(paths["mat"]), w2i, _prefix(file_name))
            if verbose:
                print("Pre-processed files don't match current settings. Reprocessing...")
        if file_name is None or not os.path.isfile(file_name):
            raise FileNotFoundError(f"[ERROR] Data file doesn't exist: {file_name}")
        if word_vec_file_name is None or not os.path.isfile(word_vec_file_name):
            raise FileNotFoundError(f"[ERROR] Word vector file doesn't exist: {word_vec_file_name}")
        with open(file_name, "r", encoding="utf-8") as f:
            ori_data = json.load(f, object_pairs_hook=OrderedDict)
        with open(word_vec_file_name, "r", encoding="utf-8") as f:
            ori_wv = json.load(f)
        word2id, mat = cls.build_word_vectors(ori_wv, case_sensitive)
        word, pos1, pos2, mask, length, r2s = cls.tensorize(ori_data, word2id, max_length, case_sensitive)
        os.makedirs(processed_dir, exist_ok=True)
        np.save(paths["word"], word)
        np.save(paths["pos1"], pos1)
        np.save(paths["pos2"], pos2)
        np.save(paths["mask"], mask)
        np.save(paths["length"], length)
        with open(paths["rel2scope"], "w") as f:
            json.dump(r2s, f)
        np.save(paths["mat"], mat)
        with open(paths["word2id"], "w") as f:
            json.dump(word2id, f)
        return cls(word, pos1, pos2, mask, length, r2s, mat, word2id, _prefix(file_name))

    @classmethod
    def from_fewrel_json_with_vocab(cls, file_name: str, word2id: Dict[str, int], word_vec_mat: np.ndarray,
                                    max_length: int, case_sensitive: bool = False) -> "FewRelDataset":
        """Tensorise a FewRel file against an existing vocabulary (no cache)."""
        with open(file_name, "r", encoding="utf-8") as f:
            ori = json.load(f, object_pairs_hook=OrderedDict)
        word, pos1, pos2, mask, length, r2s = cls.tensorize(ori, word2id, max_length, case_sensitive)
        return cls(word, pos1, pos2, mask, length, r2s, word_vec_mat, word2id, _prefix(file_name))


def truncate_word_vectors(input_file: str, output_file: str, k: int = 5) -> str:
    """The GloVe dimension-truncation tool (reference ``util/convert_glove_vec.py:3-23``):
    keep the first ``k`` dims of every vector and lower-case every word."""
    with open(input_file, "r", encoding="utf-8") as f:
        ori = json.load(f)
    out = [{"word": w["word"].lower(), "vec": w["vec"][0:k]} for w in ori]
    with open(output_file, "w", encoding="utf-8") as f:
        json.dump(out, f)
    return output_file


def vocab_from_fewrel(file_name: str, dim: int = 5, seed: int = 0, case_sensitive: bool = False) -> list:
    """Random word-vector JSON list built from the tokens of a FewRel file.

    GloVe cannot be downloaded in this environment; this gives the loader a vocabulary
    with the right format so the real ``val.json`` can be tensorised end to end."""
    with open(file_name, "r", encoding="utf-8") as f:
        ori = json.load(f, object_pairs_hook=OrderedDict)
    seen: "OrderedDict[str, None]" = OrderedDict()
    for items in ori.values():
        for ins in items:
            for t in ins["tokens"]:
                seen[t if case_sensitive else t.lower()] = None
    rng = np.random.default_rng(seed)
    vecs = rng.standard_normal((len(seen), dim)).astype(np.float32)
    return [{"word": w, "vec": [float(x) for x in v]} for w, v in zip(seen.keys(), vecs)]
