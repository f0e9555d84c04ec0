"""Label selectors (``k8s.io/apimachinery/pkg/labels`` subset).

Supports equality (``a=b`` / ``a==b``), inequality (``a!=b``), existence (``a``)
and non-existence (``!a``) requirements — what ``LabelSelectorAsSelector`` of a
``MatchLabels`` map produces (``pkg/controller/helper.go:112-119``) plus what a
``kubectl get -l`` user types.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple


class Selector:
    def __init__(self, reqs: Optional[List[Tuple[str, str, Optional[str]]]] = None):
        self.reqs = list(reqs or [])

    @classmethod
    def everything(cls) -> "Selector":
        return cls([])

    @classmethod
    def from_match_labels(cls, ml: Dict[str, str]) -> "Selector":
        return cls([(k, "=", v) for k, v in sorted(ml.items())])

    @classmethod
    def parse(cls, s: Optional[str]) -> "Selector":
        if not s:
            return cls([])
        reqs = []
        for part in s.split(","):
            part = part.strip()
            if not part:
                continue
            if "!=" in part:
                k, v = part.split("!=", 1)
                reqs.append((k.strip(), "!=", v.strip()))
            elif "==" in part:
                k, v = part.split("==", 1)
                reqs.append((k.strip(), "=", v.strip()))
            elif "=" in part:
                k, v = part.split("=", 1)
                reqs.append((k.strip(), "=", v.strip()))
            elif part.startswith("!"):
                reqs.append((part[1:].strip(), "!", None))
            else:
                reqs.append((part, "exists", None))
        return cls(reqs)

    def empty(self) -> bool:
        return not self.reqs

    def matches(self, labels: Optional[Dict[str, str]]) -> bool:
        labels = labels or {}
        for k, op, v in self.reqs:
            if op == "=":
                if labels.get(k) != v:
                    return False
            elif op == "!=":
                if labels.get(k) == v:
                    return False
            elif op == "exists":
                if k not in labels:
                    return False
            elif op == "!":
                if k in labels:
                    return False
        return True

    def __str__(self) -> str:
        out = []
        for k, op, v in self.reqs:
            if op == "exists":
                out.append(k)
            elif op == "!":
                out.append("!" + k)
            else:
                out.append(f"{k}{op}{v}")
        return ",".join(out)
