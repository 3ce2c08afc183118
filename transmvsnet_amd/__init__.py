"""transmvsnet_amd -- MI355X-native TransMVSNet depth-inference hot path (placeholder, filled below)."""
