"""Golden vectors transcribed from pkg/scheduler/framework/plugins/imagelocality/image_locality_test.go
(TestImageLocalityPriority: Score only, no NormalizeScore; TestNormalizedImageName)."""
from gen_common import case, container, node, pod

SRC = "pkg/scheduler/framework/plugins/imagelocality/image_locality_test.go"
MB = 1024 * 1024


def img(size_mb, *names):
    return {"names": list(names), "sizeBytes": size_mb * MB}


def image_pod(*images):
    return pod(containers=[container(image=i) for i in images])


NODES = {
    "node403002000": [img(40, "gcr.io/40:latest", "gcr.io/40:v1", "gcr.io/40:v1"),
                      img(300, "gcr.io/300:latest", "gcr.io/300:v1"),
                      img(2000, "gcr.io/2000:latest")],
    "node25010": [img(250, "gcr.io/250:latest"), img(10, "gcr.io/10:latest", "gcr.io/10:v1")],
    "node60040900": [img(600, "gcr.io/600:latest"), img(40, "gcr.io/40:latest"), img(900, "gcr.io/900:latest")],
    "node300600900": [img(300, "gcr.io/300:latest"), img(600, "gcr.io/600:latest"), img(900, "gcr.io/900:latest")],
    "node400030": [img(4000, "gcr.io/4000:latest"), img(30, "gcr.io/30:latest")],
    "node203040": [img(20, "gcr.io/20:latest"), img(30, "gcr.io/30:latest"), img(40, "gcr.io/40:latest")],
    "nodeWithNoImages": [],
}


def score_cases():
    out = []

    def sc(name, line, images, layout, exp):
        nodes = [node("machine%d" % (i + 1), {}, images=NODES[k]) for i, k in enumerate(layout)]
        out.append(case(name, SRC + ":%d" % line, kind="score", plugin="ImageLocality", args={},
                        pod=image_pod(*images), pods=[], nodes=nodes,
                        expect_scores={"machine%d" % (i + 1): s for i, s in enumerate(exp)}))

    sc("two images spread on two nodes, prefer the larger image one", 244,
       ["gcr.io/40", "gcr.io/250"], ["node403002000", "node25010"], [0, 5])
    sc("two images on one node, prefer this node", 259,
       ["gcr.io/40", "gcr.io/300"], ["node403002000", "node25010"], [7, 0])
    sc("if exceed limit, use limit", 274,
       ["gcr.io/10", "gcr.io/4000"], ["node400030", "node25010"], [100, 0])
    sc("if exceed limit, use limit (with node which has no images present)", 293,
       ["gcr.io/10", "gcr.io/4000"], ["node400030", "node25010", "nodeWithNoImages"], [66, 0, 0])
    sc("pod with multiple large images, machine2 is preferred", 312,
       ["gcr.io/300", "gcr.io/600", "gcr.io/900"], ["node60040900", "node300600900", "nodeWithNoImages"],
       [32, 36, 0])
    sc("pod with multiple small images", 327,
       ["gcr.io/30", "gcr.io/40"], ["node203040", "node400030"], [1, 0])
    return out


def image_name_cases():
    # TestNormalizedImageName (:356); the digest case uses the sha256 of "root", as getImageFakeDigest does
    import hashlib
    dig = "root@sha256:" + hashlib.sha256(b"root").hexdigest()
    rows = [("add :latest postfix 1", "root", "root:latest"),
            ("add :latest postfix 2", "gcr.io:5000/root", "gcr.io:5000/root:latest"),
            ("keep it as is 1", "root:tag", "root:tag"),
            ("keep it as is 2", dig, dig)]
    return [case(n, SRC + ":361", kind="image_name", input=i, expect_name=o) for n, i, o in rows]


def all_cases():
    return score_cases() + image_name_cases()
