"""MI355X-native drop-in for the ``detrex`` pieces on IR-ADS's hot path (MSDeformAttn)."""
