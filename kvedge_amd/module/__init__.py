"""IoT Edge GPU inference module: config (twin schema), transports, app."""
