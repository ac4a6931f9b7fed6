"""Model families used by the bundled TFJob payloads and the benchmark."""
