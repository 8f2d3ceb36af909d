from .schema import (  # noqa: F401
    INTENT_TYPES,
    TARGET_STRATEGIES,
    ExecuteRequest,
    Intent,
    ParseRequest,
    ParseResponse,
    SafeParseResult,
    Target,
    format_validation_error,
    safe_parse,
)
from .legacy_v0 import IntentV0, parse_intent  # noqa: F401
