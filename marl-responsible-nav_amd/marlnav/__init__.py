"""MI355X-native vectorised MARL responsible-navigation grid world (host side)."""
