"""MI355X-native drop-in for IR-ADS's ``semseg`` package (hot path: models)."""
