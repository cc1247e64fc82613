from .coco import COCOEvaluatorCustom, COCOeval, instances_to_coco_json, rle_decode, rle_encode  # noqa: F401
