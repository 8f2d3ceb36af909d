"""Legacy v0 intent shape (reference packages/schemas/src/index.ts:1-49).

Only the reference's dead CLI demo used it (apps/executor/src/index.js:3); it is kept for
API parity and so the reference's schema tests (packages/schemas/test/intent.test.ts:5-53)
have an equivalent here.
"""
from __future__ import annotations

from typing import Any, Dict, List, Literal, Optional
from urllib.parse import urlparse

from pydantic import BaseModel, Field, field_validator


class TargetV0(BaseModel):
    """packages/schemas/src/index.ts:4-10."""

    url: Optional[str] = None
    query: Optional[str] = None
    selector: Optional[str] = None
    position: Optional[Dict[str, float]] = None
    semantic: Optional[Dict[str, str]] = None

    @field_validator("url")
    @classmethod
    def _url(cls, v: Optional[str]) -> Optional[str]:
        if v is None:
            return v
        p = urlparse(v)
        if not p.scheme or not (p.netloc or p.path):
            raise ValueError("Invalid url")
        return v


class Sorting(BaseModel):
    """packages/schemas/src/index.ts:12-15."""

    field: str
    order: Literal["asc", "desc"]


class Filter(BaseModel):
    """packages/schemas/src/index.ts:17-21."""

    field: str
    op: Literal["<", "<=", "=", ">=", ">", "contains"]
    value: Any = None


class ParamsV0(BaseModel):
    value: Any = None
    filters: Optional[List[Filter]] = None
    sorting: Optional[Sorting] = None
    index: Optional[int] = Field(default=None, ge=1)
    fields: Optional[List[str]] = None
    format: Optional[Literal["csv", "json"]] = None
    filename: Optional[str] = None


class IntentV0(BaseModel):
    """packages/schemas/src/index.ts:24-42."""

    intent: str
    utterance: str
    confidence: float = Field(ge=0, le=1)
    target: Optional[TargetV0] = None
    params: Optional[ParamsV0] = None
    requires_confirmation: bool = False


def parse_intent(value: Any) -> IntentV0:
    """packages/schemas/src/index.ts:47-49 -- raises on invalid input."""
    return IntentV0.model_validate(value)
