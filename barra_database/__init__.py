"""Ingestion layer (reference: Barra_database/database/*.py): Tushare Pro -> MongoDB.

Credentials are read from the environment only (TUSHARE_TOKEN, MFA_MONGO_URI); nothing is
hard-coded (the reference embeds tokens, quirk Q24).  ``tushare`` is optional: without it (or
without a token) every fetcher returns an empty frame, as the reference does when ``pro`` is
None (tushare_fetcher.py:10-15,19).
"""
