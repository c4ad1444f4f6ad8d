"""Tiny in-memory stand-in for the pymongo surface used by the loaders/updaters (tests only)."""
import copy


def _match(doc, q):
    for k, cond in q.items():
        v = doc.get(k)
        if isinstance(cond, dict):
            for op, arg in cond.items():
                if op == "$in" and v not in arg:
                    return False
                if op == "$gte" and not (v is not None and v >= arg):
                    return False
                if op == "$lte" and not (v is not None and v <= arg):
                    return False
        elif v != cond:
            return False
    return True


class FakeCollection:
    def __init__(self):
        self.docs = []
        self.unique = None

    def find(self, query=None, projection=None):
        out = []
        for d in self.docs:
            if _match(d, query or {}):
                if projection and any(v for k, v in projection.items() if k != "_id"):
                    keep = [k for k, v in projection.items() if v and k != "_id"]
                    out.append({k: d[k] for k in keep if k in d})
                elif projection:  # exclusion-only projection, e.g. {"_id": 0}
                    drop = {k for k, v in projection.items() if not v}
                    out.append({k: v for k, v in d.items() if k not in drop})
                else:
                    out.append(copy.copy(d))
        return out

    def find_one(self, filter=None, sort=None):
        docs = [d for d in self.docs if _match(d, filter or {})]
        if sort:
            key, direction = sort[0]
            docs = sorted([d for d in docs if key in d], key=lambda d: d[key], reverse=direction < 0)
        return docs[0] if docs else None

    def insert_many(self, records, ordered=True):
        dup = 0
        for r in records:
            if self.unique:
                k = tuple(r.get(c) for c in self.unique)
                if any(tuple(d.get(c) for c in self.unique) == k for d in self.docs):
                    dup += 1
                    continue
            self.docs.append(dict(r))
        if dup:
            raise Exception(f"E11000 duplicate key error ({dup} docs)")

    def drop(self):
        self.docs = []

    def distinct(self, key):
        return sorted({d[key] for d in self.docs if key in d})


class FakeDB(dict):
    def __missing__(self, key):
        c = FakeCollection()
        self[key] = c
        return c
