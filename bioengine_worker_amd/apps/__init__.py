"""App platform: manifests, builder, service bridge, lifecycle manager."""
