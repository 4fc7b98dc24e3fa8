package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.Tags;
import org.springframework.boot.actuate.metrics.web.reactive.server.DefaultWebFluxTagsProvider;
import org.springframework.web.server.ServerWebExchange;

/**
 * The reactive (WebFlux) twin of {@link CallerTagsProvider}: the default
 * {@code http.server.requests} tags of a WebFlux server plus {@code caller},
 * the caller header's value ({@code k8s.metrics.caller-default}, "UNKNOWN",
 * when the request carries none), so the
 * downstream-impact graph (foremast_amd/engine/impact.py) also sees the
 * edges of reactive services.  An empty header name turns the tag off.
 */
public class CallerFluxTagsProvider extends DefaultWebFluxTagsProvider {

    private final String header;
    private final String absent;

    public CallerFluxTagsProvider(String header, String absent) {
        this.header = header;
        this.absent = absent == null || absent.trim().isEmpty() ? "UNKNOWN" : absent.trim();
    }

    @Override
    public Iterable<Tag> httpRequestTags(ServerWebExchange exchange, Throwable exception) {
        Tags tags = Tags.of(super.httpRequestTags(exchange, exception));
        if (header == null || header.isEmpty()) {
            return tags;
        }
        String caller = exchange == null ? null : exchange.getRequest().getHeaders().getFirst(header);
        return tags.and("caller", caller == null || caller.trim().isEmpty() ? absent : caller.trim());
    }
}
