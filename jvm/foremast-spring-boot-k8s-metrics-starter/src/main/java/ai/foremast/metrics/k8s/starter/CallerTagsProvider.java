package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.Tags;
import org.springframework.boot.actuate.metrics.web.servlet.DefaultWebMvcTagsProvider;

import javax.servlet.http.HttpServletRequest;
import javax.servlet.http.HttpServletResponse;

/**
 * {@code http.server.requests} tags plus {@code caller}: the value of the
 * caller header (X-CALLER by default), {@code k8s.metrics.caller-default}
 * ("UNKNOWN", as the reference's CallerWebMvcTagsProvider.java:14) when absent.  The brain builds its
 * downstream-impact graph from this tag (foremast_amd/engine/impact.py); an
 * empty header name turns the tag off.
 */
public class CallerTagsProvider extends DefaultWebMvcTagsProvider {

    private final String header;
    private final String absent;

    public CallerTagsProvider(String header, String absent) {
        this.header = header;
        this.absent = absent == null || absent.trim().isEmpty() ? "UNKNOWN" : absent.trim();
    }

    @Override
    public Iterable<Tag> getTags(HttpServletRequest request, HttpServletResponse response, Object handler,
                                 Throwable exception) {
        Tags tags = Tags.of(super.getTags(request, response, handler, exception));
        if (header == null || header.isEmpty()) {
            return tags;
        }
        String caller = request.getHeader(header);
        return tags.and("caller", caller == null || caller.trim().isEmpty() ? absent : caller.trim());
    }
}
