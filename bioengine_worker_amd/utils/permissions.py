"""Caller contexts and authorization (reference: bioengine/utils/permissions.py:4-104).

A context is ``{"user": {"id": ..., "email": ...}, ...}`` as injected by Hypha for services
registered with ``require_context``.  ``authorized_users``: ``"*"`` allows everyone, a user id or
email in the list allows that user, ``None``/``[]`` deny everyone.
"""
from __future__ import annotations

from typing import Any


def create_context(user_id: str | None = None, user_email: str | None = None, **extra) -> dict:
    ctx = {"user": {"id": user_id or "anonymous", "email": user_email or "anonymous@example.com"}}
    ctx.update(extra)
    return ctx


def user_identity(context: dict | None) -> tuple[str | None, str | None]:
    if not isinstance(context, dict) or not isinstance(context.get("user"), dict):
        return None, None
    u = context["user"]
    return u.get("id"), u.get("email")


def is_authorized(context: dict | None, authorized_users: Any) -> bool:
    uid, email = user_identity(context)
    if not uid and not email:
        return False
    if authorized_users in (None, [], ()):
        return False
    if isinstance(authorized_users, str):
        authorized_users = [authorized_users]
    allowed = set(authorized_users)
    return "*" in allowed or (uid is not None and uid in allowed) or (email is not None and email in allowed)


def check_permissions(context: dict | None, authorized_users: Any, resource_name: str) -> None:
    if not isinstance(context, dict) or "user" not in context:
        raise PermissionError(f"Invalid context for {resource_name}: missing user information.")
    if not isinstance(context["user"], dict):
        raise PermissionError(f"Invalid user information in context for {resource_name}.")
    uid, email = user_identity(context)
    if not uid and not email:
        raise PermissionError(f"Invalid user context for {resource_name}: need an 'id' or 'email'.")
    if authorized_users in (None, [], ()):
        raise PermissionError(f"Access denied for {resource_name}: no users are authorized.")
    if not is_authorized(context, authorized_users):
        who = f"{uid} ({email})" if email else str(uid)
        raise PermissionError(f"User {who} is not authorized to {resource_name}.")
