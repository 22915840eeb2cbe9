"""Reference-compatible import path: ``from custom.ma_customenv import CustomMAEnv``."""
