"""mtcp_amd -- MI355X-native replacement for mTCP's software checksum path."""
