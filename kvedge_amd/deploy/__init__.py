"""Deployment surface: offline Helm renderer, chart model, cloud-init, IoT Edge manifests."""
