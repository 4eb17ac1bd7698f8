"""Request schema of ``POST /response`` (reference data/requests.py:1-19)."""
from typing import List, Optional

from pydantic import BaseModel


class ChatMessage(BaseModel):
    turn: str
    message: str


class BotProfile(BaseModel):
    name: str
    appearance: str
    system_prompt: Optional[str] = ""


class UserProfile(BaseModel):
    name: str


class BotMessageRequest(BaseModel):
    bot_profile: BotProfile
    user_profile: UserProfile  # required but unused, as in the reference
    context: List[ChatMessage]
