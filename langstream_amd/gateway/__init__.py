"""langstream_amd.gateway."""
