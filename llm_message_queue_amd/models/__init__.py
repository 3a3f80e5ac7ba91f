"""Data models (C1) and the Llama-3-8B-shaped backend stub (N12)."""
from .message import (ConversationNotFound, Conversation, ConversationState, Message,
                      MessageStatus, Priority, PriorityParseError, QueueStats, LEVEL_NAMES,
                      PRIORITY_HIGH, PRIORITY_LEVELS, PRIORITY_LOW, PRIORITY_NORMAL,
                      PRIORITY_REALTIME, format_time, new_message, parse_priority, parse_time,
                      priority_name)

__all__ = [n for n in dir() if not n.startswith("_")]
