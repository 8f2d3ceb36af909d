"""Intent-parsing prompt (system rules + few-shot command set) and the Llama-3 chat layout.

Behavioural parity with the reference brain prompt (apps/brain/src/server.ts:13-82): the same
rules (JSON only, semantic targets first, wait_for when pages load, confirmation for risky
actions, follow-up question + low confidence when information is missing, short tts summary,
'unknown' when unsure, context resolution and context_updates) and the same five example
commands.  The wording is this repo's own.  The system prompt + examples form a ~1k-token static
prefix that the engine serves from the KV prefix cache (runtime/kv_cache.py).
"""
from __future__ import annotations

import json
from typing import Dict, List, Tuple

SYSTEM_PROMPT = (
    "You turn a spoken command (a speech-to-text transcript) into browser-automation intents that a "
    "headless browser will execute.\n\n"
    "Rules:\n"
    "1. Reply with JSON only, matching the intent schema exactly. Never add prose.\n"
    "2. Target elements semantically first (role and accessible name, visible text); use CSS or XPath "
    "selectors only when they are unambiguous.\n"
    "3. Add a wait_for intent whenever a step obviously has to wait for a page or a result list.\n"
    "4. Set requires_confirmation=true for anything risky: signing in, checkout or payment, entering "
    "personal data, uploading files, or destructive actions.\n"
    "5. When required details are missing, ask a follow_up_question, keep only safe intents and set "
    "confidence to 0.6 or lower.\n"
    "6. Give a short tts_summary that says, in plain language, what happens next.\n"
    "7. When you cannot tell what the user wants, emit an 'unknown' intent with confidence 0.5 or "
    "lower.\n\n"
    "Context: each request carries a small context object (current url, entity, last_intents). Use it to "
    "resolve follow-ups such as \"open the second result\", and report useful state (site, query, "
    "selected index, current url) in context_updates."
)

# (user request, assistant answer) -- the command set used by the reference few-shots and by
# the benchmark (bench.py draws its utterances from the same commands).
FEWSHOTS: List[Tuple[Dict, Dict]] = [
    (
        {"text": "search wireless earbuds", "context": {"url": "https://www.bestbuy.com", "last_intents": []}},
        {"version": "1.0", "intents": [{"type": "search", "args": {"query": "wireless earbuds"}, "priority": 0,
                                        "requires_confirmation": False}],
         "context_updates": {"query": "wireless earbuds"}, "confidence": 0.9,
         "tts_summary": "Searching for wireless earbuds.", "follow_up_question": None},
    ),
    (
        {"text": "open the second result",
         "context": {"url": "https://www.bestbuy.com/site/searchpage.jsp?st=wireless+earbuds",
                     "last_intents": [{"type": "search", "args": {"query": "wireless earbuds"}}]}},
        {"version": "1.0", "intents": [{"type": "click", "args": {},
                                        "target": {"strategy": "auto", "selector": "#search-list li:nth-of-type(2) a"},
                                        "priority": 0, "requires_confirmation": False}],
         "context_updates": {}, "confidence": 0.8, "tts_summary": "Opening the second result.",
         "follow_up_question": None},
    ),
    (
        {"text": "sort by price low to high", "context": {"entity": "bestbuy"}},
        {"version": "1.0", "intents": [{"type": "sort", "args": {"by": "price", "order": "asc"}, "priority": 0,
                                        "requires_confirmation": False}],
         "context_updates": {}, "confidence": 0.85, "tts_summary": "Sorting by lowest price.",
         "follow_up_question": None},
    ),
    (
        {"text": "upload my resume and submit the application",
         "context": {"url": "https://careers.example.com/apply",
                     "last_intents": [{"type": "navigate", "args": {"url": "https://careers.example.com/apply"}}]}},
        {"version": "1.0", "intents": [
            {"type": "upload", "args": {"fileRef": "resume://latest"},
             "target": {"strategy": "auto", "selector": "input[type=\"file\"]"}, "priority": 0,
             "requires_confirmation": True, "retries": 1},
            {"type": "click", "args": {}, "target": {"strategy": "text", "text": "Submit"}, "priority": 1,
             "requires_confirmation": True}],
         "context_updates": {}, "confidence": 0.75,
         "tts_summary": "I will upload your resume and then click submit. Please confirm.",
         "follow_up_question": None},
    ),
    (
        {"text": "search wireless earbuds and extract the top 5 with prices", "context": {"url": "https://www.bestbuy.com"}},
        {"version": "1.0", "intents": [
            {"type": "search", "args": {"query": "wireless earbuds"}, "priority": 0, "requires_confirmation": False},
            {"type": "wait_for", "args": {"selector": "[data-test=\"results\"]", "timeoutMs": 15000}, "priority": 1,
             "requires_confirmation": False},
            {"type": "extract_table", "args": {"columns": ["title", "price"], "limit": 5},
             "target": {"strategy": "auto", "selector": "[data-test=\"results\"]"}, "priority": 2,
             "requires_confirmation": False}],
         "context_updates": {"query": "wireless earbuds"}, "confidence": 0.85,
         "tts_summary": "I'll search and pull the top five items with prices.", "follow_up_question": None},
    ),
]

COMMANDS: List[str] = [u["text"] for u, _ in FEWSHOTS]

REPAIR_NOTE = ("The previous answer did not validate against the intent schema. Answer again with valid "
               "JSON only.")


def compact(obj) -> str:
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False)


def messages_for(request: Dict, repair: bool = False) -> List[Dict[str, str]]:
    """Chat messages (system, few-shots, user) -- same structure as apps/brain/src/server.ts:98-105."""
    msgs = [{"role": "system", "content": SYSTEM_PROMPT}]
    for u, a in FEWSHOTS:
        msgs.append({"role": "user", "content": compact(u)})
        msgs.append({"role": "assistant", "content": compact(a)})
    msgs.append({"role": "user", "content": compact(request)})
    if repair:
        msgs.append({"role": "system", "content": REPAIR_NOTE})
    return msgs


def llama3_chat(messages: List[Dict[str, str]]) -> Tuple[str, str]:
    """Return (static_prefix_text, dynamic_suffix_text) in the Llama-3 chat layout.

    The split point is the start of the final user turn, so the prefix is identical across
    requests and is served from the KV prefix cache.
    """
    def turn(m):
        return f"<|start_header_id|>{m['role']}<|end_header_id|>\n\n{m['content']}<|eot_id|>"

    head = "<|begin_of_text|>" + "".join(turn(m) for m in messages[:-1])
    last = messages[-1]
    tail = turn(last) + "<|start_header_id|>assistant<|end_header_id|>\n\n"
    if last["role"] == "system":  # repair note after the user turn
        head = "<|begin_of_text|>" + "".join(turn(m) for m in messages[:-2])
        tail = turn(messages[-2]) + turn(last) + "<|start_header_id|>assistant<|end_header_id|>\n\n"
    return head, tail


def plain_chat(messages: List[Dict[str, str]]) -> Tuple[str, str]:
    """(static prefix, dynamic suffix) for base LMs without chat tokens (GPT-2 config): role-tagged
    paragraphs separated by blank lines, the answer primed after ``Assistant:``."""
    def turn(m):
        return f"{m['role'].capitalize()}: {m['content']}\n\n"

    head_msgs, tail_msgs = messages[:-1], messages[-1:]
    if messages[-1]["role"] == "system":  # repair note after the user turn
        head_msgs, tail_msgs = messages[:-2], messages[-2:]
    return "".join(turn(m) for m in head_msgs), "".join(turn(m) for m in tail_msgs) + "Assistant: "


CHAT_FORMATS = {"llama3": llama3_chat, "plain": plain_chat}
