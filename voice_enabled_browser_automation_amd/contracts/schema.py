"""v1 intent contract (N5) -- pydantic v2 equivalents of the reference zod schemas.

Parity map (reference file:line):

* ``IntentType``      apps/brain/src/schema.ts:3-23  (19 values)
* ``Target``          apps/brain/src/schema.ts:25-37 (``.partial().strict().optional()``)
* ``Intent``          apps/brain/src/schema.ts:39-50 (strict; defaults args={}, priority=0,
                      requires_confirmation=false, retries=1 (0..3))
* ``ParseRequest``    apps/brain/src/schema.ts:52-58 (text min 1 "text is empty")
* ``ParseResponse``   apps/brain/src/schema.ts:60-69 (version literal "1.0", intents >= 1)
* ``ExecuteRequest``  apps/executor/src/types.ts:52-62

zod semantics reproduced here:

* ``.strict()``  -> unknown keys rejected (``extra="forbid"``).
* no type coercion: ``"true"`` is not a boolean, ``1`` is not a string, ``true`` is not a number.
* JS numbers: ``z.number().int()`` accepts ``3.0`` (an integer-valued double) -> normalised to ``3``.
* ``.partial()`` on Target means the ``strategy`` default is NOT applied when the key is absent.
* optional keys that were absent stay absent in the serialised output (``dump``), while
  defaulted keys are filled -- exactly what ``parsed.data`` looks like after zod.
"""
from __future__ import annotations

import math
from enum import Enum
from typing import Any, Dict, List, Literal, Optional

from pydantic import BaseModel, ConfigDict, Field, ValidationError, field_validator, model_validator

INTENT_TYPES: tuple[str, ...] = (
    "search",
    "navigate",
    "click",
    "type",
    "extract",
    "extract_table",
    "sort",
    "filter",
    "scroll",
    "back",
    "forward",
    "select",
    "wait_for",
    "upload",
    "screenshot",
    "summarize",
    "confirm",
    "cancel",
    "unknown",
)

TARGET_STRATEGIES: tuple[str, ...] = ("auto", "css", "text", "role", "aria", "xpath")

IntentType = Enum("IntentType", {t: t for t in INTENT_TYPES}, type=str)


def _strict_str(v: Any) -> str:
    if not isinstance(v, str):
        raise ValueError("Expected string, received " + _js_type(v))
    return v


def _strict_bool(v: Any) -> bool:
    if not isinstance(v, bool):
        raise ValueError("Expected boolean, received " + _js_type(v))
    return v


def _strict_number(v: Any) -> float:
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise ValueError("Expected number, received " + _js_type(v))
    if isinstance(v, float) and not math.isfinite(v):
        raise ValueError("Expected number, received nan")
    return v


def _strict_int(v: Any) -> int:
    v = _strict_number(v)
    if isinstance(v, float):
        if not v.is_integer():
            raise ValueError("Expected integer, received float")
        return int(v)
    return v


def _strict_record(v: Any) -> Dict[str, Any]:
    if not isinstance(v, dict):
        raise ValueError("Expected object, received " + _js_type(v))
    return v


def _js_type(v: Any) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    if isinstance(v, dict):
        return "object"
    return type(v).__name__


class _Strict(BaseModel):
    model_config = ConfigDict(extra="forbid", validate_assignment=False)

    # keys that are optional *without* a default: omitted from dump() when absent
    _omit_if_unset: tuple[str, ...] = ()

    def dump(self) -> Dict[str, Any]:
        """Serialise like zod's ``parsed.data``: defaults filled, absent optionals omitted."""
        out: Dict[str, Any] = {}
        for name in type(self).model_fields:
            if name in self._omit_if_unset and name not in self.model_fields_set:
                continue
            val = getattr(self, name)
            out[name] = _dump_value(val)
        return out


def _dump_value(val: Any) -> Any:
    if isinstance(val, _Strict):
        return val.dump()
    if isinstance(val, list):
        return [_dump_value(x) for x in val]
    if isinstance(val, dict):
        return {k: _dump_value(v) for k, v in val.items()}
    return val


class Target(_Strict):
    """apps/brain/src/schema.ts:25-37 -- every key optional (``.partial()``), strict."""

    strategy: Optional[Literal["auto", "css", "text", "role", "aria", "xpath"]] = None
    selector: Optional[str] = None
    text: Optional[str] = None
    role: Optional[str] = None
    name: Optional[str] = None

    _omit_if_unset = ("strategy", "selector", "text", "role", "name")

    @field_validator("strategy", mode="before")
    @classmethod
    def _v_strategy(cls, v: Any) -> Any:
        _strict_str(v)
        if v not in TARGET_STRATEGIES:
            raise ValueError(f"Invalid enum value. Expected {' | '.join(TARGET_STRATEGIES)}, received '{v}'")
        return v

    @field_validator("selector", "text", "role", "name", mode="before")
    @classmethod
    def _v_str(cls, v: Any) -> Any:
        return _strict_str(v)


class Intent(_Strict):
    """apps/brain/src/schema.ts:39-50."""

    type: str
    args: Dict[str, Any] = Field(default_factory=dict)
    target: Optional[Target] = None
    priority: int = 0
    requires_confirmation: bool = False
    timeout_ms: Optional[int] = None
    retries: int = 1
    clarification: Optional[str] = None

    _omit_if_unset = ("target", "timeout_ms", "clarification")

    @field_validator("type", mode="before")
    @classmethod
    def _v_type(cls, v: Any) -> Any:
        _strict_str(v)
        if v not in INTENT_TYPES:
            raise ValueError(f"Invalid enum value. Expected {' | '.join(INTENT_TYPES)}, received '{v}'")
        return v

    @field_validator("args", mode="before")
    @classmethod
    def _v_args(cls, v: Any) -> Any:
        return _strict_record(v)

    @field_validator("target", mode="before")
    @classmethod
    def _v_target(cls, v: Any) -> Any:
        if v is None:
            raise ValueError("Expected object, received null")
        return v

    @field_validator("priority", mode="before")
    @classmethod
    def _v_priority(cls, v: Any) -> Any:
        return _strict_int(v)

    @field_validator("requires_confirmation", mode="before")
    @classmethod
    def _v_rc(cls, v: Any) -> Any:
        return _strict_bool(v)

    @field_validator("timeout_ms", mode="before")
    @classmethod
    def _v_timeout(cls, v: Any) -> Any:
        v = _strict_int(v)
        if v <= 0:
            raise ValueError("Number must be greater than 0")
        return v

    @field_validator("retries", mode="before")
    @classmethod
    def _v_retries(cls, v: Any) -> Any:
        v = _strict_int(v)
        if v < 0:
            raise ValueError("Number must be greater than or equal to 0")
        if v > 3:
            raise ValueError("Number must be less than or equal to 3")
        return v

    @field_validator("clarification", mode="before")
    @classmethod
    def _v_clar(cls, v: Any) -> Any:
        return _strict_str(v)


class ParseRequest(_Strict):
    """apps/brain/src/schema.ts:52-58."""

    text: str
    session_id: Optional[str] = None
    context: Dict[str, Any] = Field(default_factory=dict)

    _omit_if_unset = ("session_id",)

    @field_validator("text", mode="before")
    @classmethod
    def _v_text(cls, v: Any) -> Any:
        _strict_str(v)
        if len(v) < 1:
            raise ValueError("text is empty")
        return v

    @field_validator("session_id", mode="before")
    @classmethod
    def _v_sid(cls, v: Any) -> Any:
        return _strict_str(v)

    @field_validator("context", mode="before")
    @classmethod
    def _v_ctx(cls, v: Any) -> Any:
        return _strict_record(v)


class ParseResponse(_Strict):
    """apps/brain/src/schema.ts:60-69."""

    version: Literal["1.0"]
    intents: List[Intent]
    context_updates: Dict[str, Any] = Field(default_factory=dict)
    confidence: float
    tts_summary: Optional[str] = None
    follow_up_question: Optional[str] = None

    _omit_if_unset = ("tts_summary", "follow_up_question")

    @field_validator("version", mode="before")
    @classmethod
    def _v_version(cls, v: Any) -> Any:
        if v != "1.0" or not isinstance(v, str):
            raise ValueError('Invalid literal value, expected "1.0"')
        return v

    @field_validator("intents", mode="before")
    @classmethod
    def _v_intents(cls, v: Any) -> Any:
        if not isinstance(v, list):
            raise ValueError("Expected array, received " + _js_type(v))
        if len(v) < 1:
            raise ValueError("Array must contain at least 1 element(s)")
        return v

    @field_validator("context_updates", mode="before")
    @classmethod
    def _v_cu(cls, v: Any) -> Any:
        return _strict_record(v)

    @field_validator("confidence", mode="before")
    @classmethod
    def _v_conf(cls, v: Any) -> Any:
        v = _strict_number(v)
        if v < 0:
            raise ValueError("Number must be greater than or equal to 0")
        if v > 1:
            raise ValueError("Number must be less than or equal to 1")
        return v

    @field_validator("tts_summary", mode="before")
    @classmethod
    def _v_tts(cls, v: Any) -> Any:
        return _strict_str(v)

    @field_validator("follow_up_question", mode="before")
    @classmethod
    def _v_fuq(cls, v: Any) -> Any:
        if v is None:
            return None
        return _strict_str(v)


class ExecuteOptions(_Strict):
    headless: Optional[bool] = None
    _omit_if_unset = ("headless",)

    @field_validator("headless", mode="before")
    @classmethod
    def _v_h(cls, v: Any) -> Any:
        return _strict_bool(v)


class ExecuteRequest(_Strict):
    """apps/executor/src/types.ts:52-62 (``options.headless`` parsed, unused as in the reference)."""

    session_id: Optional[str] = None
    intents: List[Intent]
    options: Optional[ExecuteOptions] = None

    _omit_if_unset = ("session_id", "options")

    @field_validator("session_id", mode="before")
    @classmethod
    def _v_sid(cls, v: Any) -> Any:
        return _strict_str(v)

    @field_validator("intents", mode="before")
    @classmethod
    def _v_intents(cls, v: Any) -> Any:
        if not isinstance(v, list):
            raise ValueError("Expected array, received " + _js_type(v))
        if len(v) < 1:
            raise ValueError("Array must contain at least 1 element(s)")
        return v

    @field_validator("options", mode="before")
    @classmethod
    def _v_opt(cls, v: Any) -> Any:
        if v is None:
            raise ValueError("Expected object, received null")
        return v


class SafeParseResult:
    """zod ``safeParse`` result: ``success``, ``data`` (dumped dict) or ``error``."""

    __slots__ = ("success", "data", "model", "error")

    def __init__(self, success: bool, data: Any = None, model: Any = None, error: Any = None):
        self.success = success
        self.data = data
        self.model = model
        self.error = error

    def format_error(self) -> Dict[str, Any]:
        return format_validation_error(self.error)


def safe_parse(model_cls: type[_Strict], value: Any) -> SafeParseResult:
    if not isinstance(value, dict):
        err = ValueError("Expected object, received " + _js_type(value))
        return SafeParseResult(False, error=err)
    try:
        m = model_cls.model_validate(value)
    except ValidationError as e:
        return SafeParseResult(False, error=e)
    return SafeParseResult(True, data=m.dump(), model=m)


def format_validation_error(err: Any) -> Dict[str, Any]:
    """Shape errors like zod's ``error.format()``: nested ``{_errors: [...], key: {...}}``."""
    root: Dict[str, Any] = {"_errors": []}
    if isinstance(err, ValidationError):
        for e in err.errors():
            node = root
            for loc in e["loc"]:
                key = str(loc)
                node = node.setdefault(key, {"_errors": []})
            msg = e.get("msg", "invalid")
            if msg.startswith("Value error, "):
                msg = msg[len("Value error, ") :]
            if e.get("type") == "extra_forbidden":
                msg = "Unrecognized key(s) in object"
            elif e.get("type") == "missing":
                msg = "Required"
            node["_errors"].append(msg)
    elif err is not None:
        root["_errors"].append(str(err))
    return root
