"""MI355X-native drop-in for IR-ADS's ``modules`` package (LightSB)."""
