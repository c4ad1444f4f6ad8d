"""Configuration, IO, logging, timing and checkpoint utilities."""
